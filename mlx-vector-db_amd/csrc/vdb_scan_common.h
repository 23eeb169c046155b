// vdb_scan_common.h — device pieces shared by the candidate-pass kernels (vdb_scan.hip: the
// fp32 pass; vdb_scan2.hip: the split-bf16 passes): per-query LDS top-KP compaction, the
// XCD-aware block mapping, the flush of surviving candidates to the global per-query lists.
#pragma once
#include "vdb_common.h"

namespace vdb {

// Compaction of one query's append buffer (one wave): keep the best KP entries
// by (score desc, row asc), unsorted, in slots [0, KP); the threshold becomes the
// KP-th best score.  Selection is a bisection over the order-preserving score
// bits with wave ballots (then over row ids among ties at the threshold), so a
// compaction costs ~32 ballot rounds instead of a sort network.
template <int KP, int CAP>
__device__ __forceinline__ void compact_query(float* sc, uint32_t* ix, int* cnt, float* thr, uint32_t* gslot) {
    constexpr int E = (CAP + 63) / 64;  // CAP need not be a multiple of 64 (scan3: 48)
    const int lane = threadIdx.x & 63;
    const int n = *cnt < CAP ? *cnt : CAP;
    if (n <= KP) return;
    float sv[E];
    uint32_t kv[E], iv[E];
    bool ok[E];
#pragma unroll
    for (int i = 0; i < E; ++i) {
        const int e = i * 64 + lane;
        ok[i] = e < n;
        sv[i] = ok[i] ? sc[e] : 0.0f;
        iv[i] = ok[i] ? ix[e] : 0xFFFFFFFFu;
        kv[i] = order_key(sv[i]);
    }
    uint32_t T = 0;
    for (int bit = 31; bit >= 0; --bit) {
        const uint32_t c = T | (1u << bit);
        int n_ge = 0;
#pragma unroll
        for (int i = 0; i < E; ++i) n_ge += __popcll(__ballot(ok[i] && kv[i] >= c));
        if (n_ge >= KP) T = c;
    }
    int c_gt = 0, c_eq = 0;
#pragma unroll
    for (int i = 0; i < E; ++i) {
        c_gt += __popcll(__ballot(ok[i] && kv[i] > T));
        c_eq += __popcll(__ballot(ok[i] && kv[i] == T));
    }
    const int need = KP - c_gt;  // >= 1 of the ties, lowest rows first
    uint32_t I = 0xFFFFFFFFu;
    if (c_eq > need) {
        I = 0;
        for (int bit = 31; bit >= 0; --bit) {
            const uint32_t c = I | (1u << bit);
            int n_lt = 0;
#pragma unroll
            for (int i = 0; i < E; ++i) n_lt += __popcll(__ballot(ok[i] && kv[i] == T && iv[i] < c));
            if (n_lt < need) I = c;
        }
    }
    int base = 0;
#pragma unroll
    for (int i = 0; i < E; ++i) {
        const bool keep = ok[i] && (kv[i] > T || (kv[i] == T && iv[i] <= I));
        const unsigned long long b = __ballot(keep);
        const int pos = base + __popcll(b & ((1ull << lane) - 1ull));
        base += __popcll(b);
        if (keep) {
            sc[pos] = sv[i];
            ix[pos] = iv[i];
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (lane == 0) {
        const uint32_t u = (T & 0x80000000u) ? (T & 0x7FFFFFFFu) : ~T;
        *thr = __uint_as_float(u);
        *cnt = KP;
        // publish: this workgroup's KP-th best is a lower bound of the global KP-th best
        if (gslot) atomicMax(gslot, T);
    }
}


typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// Corpus stream loads.  With one query block (B <= 64) every corpus byte is read
// once per launch: the non-temporal policy (global_load_dwordx4 ... nt) then gives
// C2 587 -> 559 us.  With several query blocks the blocks of one row range share
// its lines through the XCD's L2 (xcd_map), which nt defeats (C3 2.62 -> 3.12 ms,
// C4 7.56 -> 8.89 ms): default policy there.  Measured A/B on MI355X.
// Operand planes per precision: XPL corpus planes loaded per group, QPL query
// planes, LPL planes in the corpus layout (the split layout holds hi and lo).
//   PREC_FP32    fp32 x fp32                  XPL 1  QPL 1  LPL 1
//   PREC_BF16X3  (xh + xl) x (qh + ql)        XPL 2  QPL 2  LPL 2
//   PREC_BF16    xh x (qh + ql): half the corpus bytes of the other two
template <int PREC>
struct Planes {
    static constexpr int XPL = PREC == PREC_BF16X3 ? 2 : 1;
    static constexpr int QPL = PREC == PREC_FP32 ? 1 : 2;
    static constexpr int LPL = PREC == PREC_FP32 ? 1 : 2;
};

template <bool NT>
__device__ __forceinline__ f32x4 corpus_ld(const float* p) {
    if constexpr (NT) return __builtin_nontemporal_load((const f32x4*)p);
    else return *(const f32x4*)p;
}

// 1-D grid of round_up(n_wg, 8) * n_qb workgroups -> (row range wg, query block qb):
// block L sits on XCD L % 8; ranges wg = 8 (j / n_qb) + L % 8 with j = L / 8, so the
// n_qb blocks of a range share an XCD and consecutive dispatch slots.  Ranges past
// n_wg get no steps (s_begin >= n_steps) and only flush nothing.
__device__ __forceinline__ void xcd_map(int n_qb, int& wg, int& qb) {
    const int L = blockIdx.x;
    const int j = L >> 3;
    qb = j % n_qb;
    wg = (j / n_qb) * 8 + (L & 7);
}

// Flush of one wave's queries q(i) = q0 + qstep i (i < nq <= 64): the entries of LDS
// buffer q (CAPX slots, cnt[q] used) scoring above that query's bound T (order key in
// lane i's `tkey`) are appended to the global list of query qb0 + q.  One returning
// atomic per query, all issued together (lane i for query i), so the flush costs one
// round trip, not nq of them.
template <int CAPX>
__device__ __forceinline__ void append_flush(const float* sc, const uint32_t* ix, const int* cnt, int q0, int qstep,
                                             int nq, int qb0, int B, uint32_t tkey, float* __restrict__ gl_s,
                                             uint32_t* __restrict__ gl_i, uint32_t* __restrict__ gl_cnt,
                                             int64_t gl_cap) {
    constexpr int EW = (CAPX + 63) / 64;
    const int lane = threadIdx.x & 63;
    int myc = 0;
    for (int i = 0; i < nq; ++i) {
        const int q = q0 + qstep * i;
        const float Tq = key_to_float((uint32_t)__shfl((int)tkey, i, 64));
        const int n = min(cnt[q], CAPX);
        int c = 0;
#pragma unroll
        for (int j = 0; j < EW; ++j) {
            const int e = j * 64 + lane;
            c += __popcll(__ballot(e < n && sc[q * CAPX + e] > Tq));
        }
        if (lane == i) myc = c;
    }
    int mybase = 0;
    if (lane < nq && qb0 + q0 + qstep * lane < B && myc > 0)
        mybase = (int)atomicAdd(gl_cnt + qb0 + q0 + qstep * lane, (uint32_t)myc);
    for (int i = 0; i < nq; ++i) {
        const int q = q0 + qstep * i;
        const int qg = qb0 + q;
        if (qg >= B) continue;
        const float Tq = key_to_float((uint32_t)__shfl((int)tkey, i, 64));
        const int n = min(cnt[q], CAPX);
        int base = __shfl(mybase, i, 64);
#pragma unroll
        for (int j = 0; j < EW; ++j) {
            const int e = j * 64 + lane;
            const bool pass = e < n && sc[q * CAPX + e] > Tq;
            const unsigned long long m = __ballot(pass);
            const int64_t pos = (int64_t)base + __popcll(m & ((1ull << lane) - 1ull));
            if (pass && pos < gl_cap) {
                gl_s[(size_t)qg * gl_cap + pos] = sc[q * CAPX + e];
                gl_i[(size_t)qg * gl_cap + pos] = ix[q * CAPX + e];
            }
            base += __popcll(m);
        }
    }
}

// Inner products of one 8-dim (fp32) or 16-dim (split-bf16) group of RT corpus
// tiles against QT query tiles.  PREC_BF16X3: x.q ~ xh.qh + xh.ql + xl.qh, each
// product exact in fp32, dropped terms <= ~3 2^-16 |x||q| per element; PREC_BF16:
// x.q ~ xh.qh + xh.ql, off by |x - xh| <= 2^-9 |x| per element.
template <int PREC, int RT, int QT>
__device__ __forceinline__ void group_mfma(const f32x4 (&x)[RT][Planes<PREC>::XPL],
                                           const f32x4 (&q)[QT][Planes<PREC>::QPL], f32x16 (&acc)[RT][QT]) {
    if constexpr (PREC == PREC_FP32) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int qt = 0; qt < QT; ++qt)
                    acc[rt][qt] = __builtin_amdgcn_mfma_f32_32x32x2f32(x[rt][0][j], q[qt][0][j], acc[rt][qt], 0, 0, 0);
    } else if constexpr (PREC == PREC_BF16) {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int qt = 0; qt < QT; ++qt) {
                const bf16x8 xh = __builtin_bit_cast(bf16x8, x[rt][0]);
                const bf16x8 qh = __builtin_bit_cast(bf16x8, q[qt][0]), ql = __builtin_bit_cast(bf16x8, q[qt][1]);
                acc[rt][qt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xh, ql, acc[rt][qt], 0, 0, 0);
                acc[rt][qt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xh, qh, acc[rt][qt], 0, 0, 0);
            }
    } else {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int qt = 0; qt < QT; ++qt) {
                const bf16x8 xh = __builtin_bit_cast(bf16x8, x[rt][0]), xl = __builtin_bit_cast(bf16x8, x[rt][1]);
                const bf16x8 qh = __builtin_bit_cast(bf16x8, q[qt][0]), ql = __builtin_bit_cast(bf16x8, q[qt][1]);
                acc[rt][qt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xl, qh, acc[rt][qt], 0, 0, 0);
                acc[rt][qt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xh, ql, acc[rt][qt], 0, 0, 0);
                acc[rt][qt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xh, qh, acc[rt][qt], 0, 0, 0);
            }
    }
}

}  // namespace vdb
