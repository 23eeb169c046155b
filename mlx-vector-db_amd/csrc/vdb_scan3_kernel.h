// vdb_scan3_kernel.h — the large-batch split-bf16 candidate pass (B >= 128 queries: C3's 256,
// C4's 512).  Same arithmetic, inputs and outputs as scan2 (vdb_scan2_kernel.h), the other
// loop shape:
//
//   scan2: the 4 waves of a workgroup share one query block (64 queries) and stream different
//          rows, each wave loading its own corpus tiles and re-loading the query tiles; several
//          query blocks re-read every row range through the XCD's L2.
//   scan3: the 4 waves share the ROWS: each group of RT row tiles (RT x 32 rows x 16 dims,
//          both planes for bf16x3) is loaded once per workgroup (register-staged, one 1 KiB
//          piece per lane-load) into a double-buffered LDS slot, and every wave multiplies it
//          against ITS OWN 2 query tiles (64 queries), so one workgroup covers 256 queries
//          and the corpus is read once per 256 queries.
//
// Bytes from L2 per group and CU (bf16, RT = 8): 8 KiB of rows + 4 x 4 KiB of query tiles for
// 4 x 32 MFMAs (1024 cycles per SIMD): 24 B/clk, under the ~30 B/clk an L2-fed CU sustains
// (MI355X_MICROARCH.md, gather from L2); scan2 at C3 needs 20 KiB per 512 cycles (40 B/clk).
//
// Top-k: each wave owns its 64 queries, so their LDS candidate buffers are wave-private (no
// workgroup barrier, no LDS atomics across waves).  A buffer keeps the best KW (< KP) of the
// rows its workgroup saw; when it compacts, its KW-th best becomes the workgroup's drop bound
// for that query, which the flush raises gthr to.  The certificate's invariant (vdb_exact.hip
// finish: every row outside the final list scored <= max(a_KP, gthr)) holds as for scan2; a
// workgroup holding more than KW of a query's true top k only costs that query the exact
// fallback, so scan3 is used where rows per workgroup >> KP (vdb_api.cpp).
#pragma once
#include "vdb_common.h"
#include "vdb_internal.h"
#include "vdb_scan_common.h"

namespace vdb {

constexpr int S3_NW = 4;   // waves per workgroup (one per SIMD)
constexpr int S3_QTW = 2;  // query tiles per wave
constexpr int S3_QB = S3_NW * S3_QTW * 32;  // queries per workgroup block (256)
#ifndef VDB_S3_RT
#define VDB_S3_RT 8
#endif
constexpr int S3_RT = VDB_S3_RT;          // row tiles per step, shared by the waves
constexpr int S3_ROWS = S3_RT * 32;       // rows per step

// row-valid bits of row tile t for this lane (as scan2's tile_valid16)
__device__ __forceinline__ uint32_t s3_valid16(const uint32_t* mask, int64_t t, int64_t N, int lane) {
    uint32_t w = 0xFFFFFFFFu;
    if (mask) w = t < ((N + 31) >> 5) ? mask[t] : 0u;
    const int64_t rem = N - t * 32;
    if (rem < 32) w &= rem <= 0 ? 0u : ((1u << rem) - 1u);
    w >>= 4 * (lane >> 5);
    return (w & 0xFu) | ((w >> 4) & 0xF0u) | ((w >> 8) & 0xF00u) | ((w >> 12) & 0xF000u);
}

__device__ __forceinline__ float s3_max16(const f32x16& a) {
    float m = __builtin_elementwise_maximum(__builtin_elementwise_maximum(a[0], a[1]), a[2]);
#pragma unroll
    for (int v = 3; v < 15; v += 2) m = __builtin_elementwise_maximum(__builtin_elementwise_maximum(m, a[v]), a[v + 1]);
    return __builtin_elementwise_maximum(m, a[15]);
}

// PREC: PREC_BF16 / PREC_BF16X3; KW kept per query and workgroup, CAP buffer slots; RING
// corpus register sets in flight (loads issued RING groups ahead of their LDS write); PQ query
// groups in flight; GC > 0: the group count as a compile-time constant (short rows, C4: 8).
template <int PREC, int METRIC, int KW, int CAP, int RING, int PQ, int GC>
__global__ void __launch_bounds__(64 * S3_NW, 1)
scan3_kernel(const float* __restrict__ Xs, const float* __restrict__ rinit, const uint32_t* __restrict__ mask,
             const float* __restrict__ Qs, int G_arg, int64_t N, int B, int64_t n_steps, int steps_per_wg, int n_qb,
             float* __restrict__ gl_s, uint32_t* __restrict__ gl_i, uint32_t* __restrict__ gl_cnt, int64_t gl_cap,
             uint32_t* __restrict__ gthr) {
    constexpr int RT = S3_RT, NW = S3_NW, QT = S3_QTW;
    constexpr int XPL = Planes<PREC>::XPL;
    constexpr int PIECES = RT * XPL;        // 1 KiB pieces per group
    constexpr int PPW = PIECES / NW;        // pieces per wave
    static_assert(PIECES % NW == 0, "corpus pieces per group must split over the waves");
    static_assert(PQ <= QG_EXTRA, "query prefetch deeper than the duplicated groups");
    constexpr size_t GSTEP = 8 * BLOCK_FLOATS;  // query: consecutive groups of one super tile
    constexpr size_t PLANE = 4 * BLOCK_FLOATS;  // query: lo plane after hi
    const int G = GC > 0 ? GC : G_arg;
    const size_t XPLANE = corpus_plane(G);

    __shared__ __attribute__((aligned(16))) float s_x[2][PIECES * 256];  // corpus slots (group parity)
    __shared__ float s_sc[NW][64 * CAP];
    __shared__ uint32_t s_ix[NW][64 * CAP];
    __shared__ int s_cnt[NW][64];
    __shared__ float s_thr[NW][64];

    const int lane = threadIdx.x & 63;
    const int lane4 = lane * 4;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int wg, qb;
    xcd_map(n_qb, wg, qb);
    const int q0 = qb * S3_QB + wv * 64;  // this wave's first query
    s_cnt[wv][lane] = 0;
    s_thr[wv][lane] = -INFINITY;

    const int64_t s_begin = (int64_t)wg * steps_per_wg;
    const int64_t s_end = s_begin + steps_per_wg < n_steps ? s_begin + steps_per_wg : n_steps;
    const int64_t n_grp = (s_end > s_begin ? s_end - s_begin : 0) * G;  // groups this workgroup runs

    // corpus piece p of linear group u (u = step * G + g): plane p / RT, row tile p % RT
    auto piece_src = [&](int64_t u, int p) -> const float* {
        if (u >= n_grp) u = n_grp - 1;  // prefetch past the end: re-read the last group (unused)
        const int64_t s = s_begin + u / G;
        const int g = (int)(u % G);
        return Xs + corpus_block((uint64_t)(s * RT + p % RT), g, 0, G) + (size_t)(p / RT) * XPLANE + lane4;
    };
    // register rings (creg: corpus pieces of groups u+1 .. u+RING; qreg: query tiles of groups
    // u .. u+PQ-1) indexed by compile-time slots only: the rings shift by one each group (register
    // moves), a runtime slot index would put them in scratch memory
    f32x4 creg[RING][PPW];
    auto cload = [&](int slot, int64_t u) {
#pragma unroll
        for (int j = 0; j < PPW; ++j) creg[slot][j] = *(const f32x4*)piece_src(u, wv + NW * j);
    };
    auto cstore = [&](int slot, int buf) {
#pragma unroll
        for (int j = 0; j < PPW; ++j) *(f32x4*)(&s_x[buf][(wv + NW * j) * 256 + lane4]) = creg[slot][j];
    };
    auto cshift = [&]() {
#pragma unroll
        for (int r = 0; r + 1 < RING; ++r)
#pragma unroll
            for (int j = 0; j < PPW; ++j) creg[r][j] = creg[r + 1][j];
    };
    const float* Qw = Qs + split_block((uint64_t)(q0 / 32), 0, G + QG_EXTRA);  // the wave's 2 tiles (one super tile)
    f32x4 qreg[PQ][QT][2];
    const bool qlive = q0 < B;  // (Qs holds round_up(B, 128) queries: waves past B load nothing)
    auto qload = [&](int slot, int g) {
        if (!qlive) return;
#pragma unroll
        for (int qt = 0; qt < QT; ++qt)
#pragma unroll
            for (int pl = 0; pl < 2; ++pl)
                qreg[slot][qt][pl] = *(const f32x4*)(Qw + (size_t)g * GSTEP + pl * PLANE + qt * BLOCK_FLOATS + lane4);
    };

    const bool active = n_grp > 0 && q0 < B;  // wave-uniform; whole workgroups share n_grp
    if (n_grp > 0) {
        // prologue: group 0 into LDS slot 0; groups 1 .. RING in the corpus ring; query groups
        // 0 .. PQ-1 in the query ring
        cload(0, 0);
        cstore(0, 0);
#pragma unroll
        for (int r = 0; r < RING; ++r) cload(r, r + 1);
#pragma unroll
        for (int p = 0; p < PQ; ++p) qload(p, p);
    }
    __syncthreads();

    const float ones = lane < 32 ? 1.0f : 0.0f;
    int64_t u = 0;  // linear group
    for (int64_t s = s_begin; s < s_end; ++s) {
        const int64_t t0 = s * RT;  // first row tile of the step
        f32x16 acc[RT][QT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            float r1 = 0.0f;
            if constexpr (METRIC == 1) r1 = lane < 32 ? rinit[(t0 + rt) * 32 + lane] : 0.0f;
#pragma unroll
            for (int qt = 0; qt < QT; ++qt) {
#pragma unroll
                for (int v = 0; v < 16; ++v) acc[rt][qt][v] = 0.0f;
                if constexpr (METRIC == 1)  // acc[i][j] = rinit[row i] (exact), as scan2
                    acc[rt][qt] = __builtin_amdgcn_mfma_f32_32x32x2f32(r1, ones, acc[rt][qt], 0, 0, 0);
            }
        }
        uint32_t gk[QT];
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
            const int qg = q0 + qt * 32 + (lane & 31);
            gk[qt] = qg < B ? gthr[qg] : 0u;
        }
        for (int g = 0; g < G; ++g, ++u) {
            const int buf = (int)(u & 1);
            // group u+1 into the other slot (its last readers, group u-1, are past the barrier
            // that ended the previous group); the ring shifts and loads group u+1+RING
            if (u + 1 < n_grp) {
                cstore(0, buf ^ 1);
                cshift();
                cload(RING - 1, u + 1 + RING);
            }
            // MFMAs of group u: A = the shared row tiles from LDS, B = this wave's query tiles
            f32x4 qb_[QT][2];
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                for (int pl = 0; pl < 2; ++pl) {
                    qb_[qt][pl] = qreg[0][qt][pl];
#pragma unroll
                    for (int r = 0; r + 1 < PQ; ++r) qreg[r][qt][pl] = qreg[r + 1][qt][pl];
                }
            qload(PQ - 1, g + PQ);  // duplicated groups cover g + PQ >= G (the next step's)
            if (active) {
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) {
                    f32x4 xa[1][XPL];
#pragma unroll
                    for (int pl = 0; pl < XPL; ++pl) xa[0][pl] = *(const f32x4*)(&s_x[buf][(pl * RT + rt) * 256 + lane4]);
                    f32x16 a2[1][QT];
#pragma unroll
                    for (int qt = 0; qt < QT; ++qt) a2[0][qt] = acc[rt][qt];
                    group_mfma<PREC, 1, QT>(xa, qb_, a2);
#pragma unroll
                    for (int qt = 0; qt < QT; ++qt) acc[rt][qt] = a2[0][qt];
                }
            }
            __syncthreads();
        }
        if (!active) continue;
#ifdef VDB_S3_KLOOP_ONLY
        {  // diagnostic build: the K-loop alone, results are garbage
            float f = 0.0f;
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int qt = 0; qt < QT; ++qt) f += s3_max16(acc[rt][qt]);
            if (f == 1234.5f) gl_s[0] = f;
            continue;
        }
#endif
        // ---- epilogue: the accumulators are the scores (cosine) or half of them (L2) ----
        float thrh[QT];
        bool qok[QT];
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
            const int ql = qt * 32 + (lane & 31);
            const float thr = fmaxf(s_thr[wv][ql], key_to_float(gk[qt]));
            thrh[qt] = METRIC == 0 ? thr : 0.5f * thr;
            qok[qt] = q0 + ql < B;
        }
        auto insert_pass = [&](int rt, int qt, float th, uint32_t cand) -> uint32_t {
            const int ql = qt * 32 + (lane & 31);
            uint32_t left = 0;
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                const bool p = ((cand >> v) & 1u) && acc[rt][qt][v] > th;
                if (__any(p)) {
                    if (p) {
                        float a_ = acc[rt][qt][v];
                        uint32_t rb = (uint32_t)((t0 + rt) * 32) + 4u * (uint32_t)(lane >> 5);
                        asm volatile("" : "+v"(a_), "+v"(rb));
                        const float sc = METRIC == 0 ? a_ : 2.0f * a_;
                        const int pos = atomicAdd(&s_cnt[wv][ql], 1);
                        if (pos < CAP) {
                            s_sc[wv][ql * CAP + pos] = sc;
                            s_ix[wv][ql * CAP + pos] = rb + (uint32_t)((v & 3) + 8 * (v >> 2));
                        } else {
                            left |= 1u << v;
                        }
                    }
                }
            }
            return left;
        };
        uint32_t pend[RT][QT];
        uint32_t any_left = 0;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int qt = 0; qt < QT; ++qt) {
                pend[rt][qt] = 0u;
                if (__any(qok[qt] && s3_max16(acc[rt][qt]) > thrh[qt])) {
                    const uint32_t valid = qok[qt] ? s3_valid16(mask, t0 + rt, N, lane) : 0u;
                    pend[rt][qt] = insert_pass(rt, qt, thrh[qt], valid);
                    any_left |= pend[rt][qt];
                }
            }
        // full buffers: compact them (this wave's queries only, no workgroup barrier) and retry
        while (__any(any_left != 0)) {
            for (int q = 0; q < 64; ++q)
                if (s_cnt[wv][q] >= CAP)
                    compact_query<KW, CAP>(s_sc[wv] + q * CAP, s_ix[wv] + q * CAP, &s_cnt[wv][q], &s_thr[wv][q],
                                           nullptr);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            any_left = 0;
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int qt = 0; qt < QT; ++qt) {
                    if (!__any(pend[rt][qt] != 0)) continue;
                    const int ql = qt * 32 + (lane & 31);
                    const float thr = fmaxf(s_thr[wv][ql], key_to_float(gk[qt]));
                    pend[rt][qt] = insert_pass(rt, qt, METRIC == 0 ? thr : 0.5f * thr, pend[rt][qt]);
                    any_left |= pend[rt][qt];
                }
        }
    }

    // ---- flush: this wave's 64 queries ----
    if (n_grp > 0 && q0 < B) {
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        // a compacted buffer dropped rows at or below its KW-th best: raise gthr to it (the
        // certificate's bound), then append the entries above max(gthr, that bound)
        const int qg = q0 + lane;
        uint32_t tkey = 0;
        if (qg < B) {
            const float th = s_thr[wv][lane];
            const uint32_t dk = th == -INFINITY ? 0u : order_key(th);
            if (dk) atomicMax(gthr + qg, dk);
            tkey = max(gthr[qg], dk);
        }
        append_flush<CAP>(s_sc[wv], s_ix[wv], s_cnt[wv], 0, 1, 64, q0, B, tkey, gl_s, gl_i, gl_cnt, gl_cap);
    }
}


template <int P, int M, int KW, int CAP, int RING, int PQ, int GC>
static hipError_t scan3_launch_g(const float* Xs, const float* rinit, const uint32_t* mask, const float* Qs, int G,
                                 int64_t N, int B, int n_qblocks, int64_t n_steps, int n_wg, int spw, float* gl_s,
                                 uint32_t* gl_i, uint32_t* gl_cnt, int64_t gl_cap, uint32_t* gthr, hipStream_t st) {
    const int n_wg8 = (n_wg + 7) / 8 * 8;
    hipLaunchKernelGGL((scan3_kernel<P, M, KW, CAP, RING, PQ, GC>), dim3(n_wg8 * n_qblocks), dim3(64 * S3_NW), 0, st,
                       Xs, rinit, mask, Qs, G, N, B, n_steps, spw, n_qblocks, gl_s, gl_i, gl_cnt, gl_cap, gthr);
    return hipGetLastError();
}

#define S3_UNIT_PARAMS                                                                                         \
    const float *Xs, const float *rinit, const uint32_t *mask, const float *Qs, int G, int64_t N, int B,        \
        int n_qblocks, int64_t n_steps, int n_wg, int spw, float *gl_s, uint32_t *gl_i, uint32_t *gl_cnt,      \
        int64_t gl_cap, uint32_t *gthr, hipStream_t st
// register sets of corpus pieces in flight (groups ahead of their LDS write): bf16 3 (2 pieces
// per wave and set), bf16x3 2 (4 pieces); query groups in flight 2
#ifndef VDB_S3_RING_2
#define VDB_S3_RING_2 3
#endif
#ifndef VDB_S3_RING_1
#define VDB_S3_RING_1 2
#endif
#ifndef VDB_S3_PQ
#define VDB_S3_PQ 2
#endif
#define S3_ARGS Xs, rinit, mask, Qs, G, N, B, n_qblocks, n_steps, n_wg, spw, gl_s, gl_i, gl_cnt, gl_cap, gthr, st
// One instantiation unit per (precision, metric): KW = 32 kept per query and workgroup
// (CAP 48), the short-row (D = 128, 8 groups) case with the group count built in.
#define S3_UNIT(NAME, P, M, RINGV, PQV)                                                    \
    hipError_t NAME(S3_UNIT_PARAMS) {                                                     \
        if (G == 8) return scan3_launch_g<P, M, 32, 48, RINGV, PQV, 8>(S3_ARGS);          \
        return scan3_launch_g<P, M, 32, 48, RINGV, PQV, 0>(S3_ARGS);                      \
    }
hipError_t launch_scan3_b3c(S3_UNIT_PARAMS);
hipError_t launch_scan3_b3l(S3_UNIT_PARAMS);
hipError_t launch_scan3_b1c(S3_UNIT_PARAMS);
hipError_t launch_scan3_b1l(S3_UNIT_PARAMS);

}  // namespace vdb
