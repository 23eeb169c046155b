// vdb_scan.hip — gfx950 kernels of the brute-force distance + top-k path.
//
// Pipeline for one search:
//   prep_queries  -> scan_topk (fp32 MFMA candidate pass, fused per-WG top-KP)
//   -> merge_lists (per-query top-KP over all WG lists)
//   -> rerank (exact fp64 keys of the KP candidates, top-k, certificate)
//   -> [rare] exact_scan + merge + finalize for queries whose certificate failed.
//
// Reference semantics restated here (file:line in /root/reference):
//   cosine  = (q/max(|q|,1e-8)).(x/max(|x|,1e-8))   service/optimized_vector_store.py:31-41
//   L2      = sqrt(sum((x-q)^2))                    service/optimized_vector_store.py:43-48
//   order   = argsort(-score)[:k] / argsort(dist)[:k], ties -> lower row
//                                                   service/optimized_vector_store.py:176-183
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off (fp64 canonical order).
#include "vdb_common.h"
#include "vdb_internal.h"

namespace vdb {

#ifdef VDB_STAMP
// Diagnostic build only (make stamp): per-wave cycle counters of the scan
// kernel; never compiled into the product library.
__device__ unsigned long long g_scan_stamps[1 << 16][8];
#define STAMP_NOW() __builtin_amdgcn_s_memtime()
#endif

// =============================================================================
// Candidate pass: fp32 MFMA scores fused with a per-workgroup top-KP
// =============================================================================
// Workgroup = 4 waves.  Wave w of step s owns row tiles (4 s + w) RT .. +RT-1
// (RT*32 rows) and all QB = 32 QT queries of its query block.  Per 8-dim group
// it issues RT + QT global_load_dwordx4 (corpus from HBM, queries from L2) and
// 4 RT QT v_mfma_f32_32x32x2_f32.  Corpus loads run PX groups ahead and query
// loads PQ groups ahead, in registers: the corpus operand is streamed once and
// not shared across waves, so it does not go through LDS.
// Accumulator lane l / register v holds query 32 qt + (l & 31) against corpus
// row 32 t + (v & 3) + 8 (v >> 2) + 4 (l >> 5).
//
// Top-KP per query lives in LDS: an append buffer of CAP = 2 KP (4 KP for
// KP = 32: fewer compaction rounds while the first step fills it) (score, row)
// per query plus a threshold (the KP-th best after the last compaction).  A
// score enters only if it beats the threshold; when a buffer fills, one wave
// selects the best KP by bisection (compact_query).  Invariant used by the certificate in
// rerank: every row not in the final list scored <= the list's KP-th entry.
__device__ __forceinline__ uint32_t order_key(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);  // float order -> unsigned order
}

// Compaction of one query's append buffer (one wave): keep the best KP entries
// by (score desc, row asc), unsorted, in slots [0, KP); the threshold becomes the
// KP-th best score.  Selection is a bisection over the order-preserving score
// bits with wave ballots (then over row ids among ties at the threshold), so a
// compaction costs ~32 ballot rounds instead of a sort network.
template <int KP, int CAP>
__device__ __forceinline__ void compact_query(float* sc, uint32_t* ix, int* cnt, float* thr, uint32_t* gslot) {
    constexpr int E = CAP / 64;
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

__device__ __forceinline__ float key_to_float(uint32_t k) {
    if (k == 0) return -INFINITY;
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

// Final per-query list: best min(n, KP) entries sorted, sentinel padded.
template <int KP, int CAP>
__device__ __forceinline__ void flush_query(float* sc, uint32_t* ix, int* cnt, float* thr, float* out_s,
                                            uint32_t* out_i) {
    constexpr int EK = KP >= 64 ? KP / 64 : 1;
    const int lane = threadIdx.x & 63;
    compact_query<KP, CAP>(sc, ix, cnt, thr, nullptr);
    const int n = *cnt < KP ? *cnt : KP;
    float sv[EK];
    uint32_t iv[EK];
#pragma unroll
    for (int i = 0; i < EK; ++i) {
        const int e = i * 64 + lane;
        sv[i] = e < n ? sc[e] : -INFINITY;
        iv[i] = e < n ? ix[e] : 0xFFFFFFFFu;
    }
    wave_sort_desc<float, uint32_t, EK>(sv, iv);
    if (out_s) {
#pragma unroll
        for (int i = 0; i < EK; ++i) {
            const int e = i * 64 + lane;
            if (e < KP) {
                out_s[e] = sv[i];
                out_i[e] = iv[i];
            }
        }
    }
}

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// Inner products of one 8-dim (fp32) or 16-dim (split-bf16) group of RT corpus
// tiles against QT query tiles.  PREC_BF16X3: x.q ~ xh.qh + xh.ql + xl.qh, each
// product exact in fp32, dropped terms <= ~3 2^-16 |x||q| per element.
template <int PREC, int RT, int QT>
__device__ __forceinline__ void group_mfma(const f32x4 (&x)[RT][PREC + 1], const f32x4 (&q)[QT][PREC + 1],
                                           f32x16 (&acc)[RT][QT]) {
    if constexpr (PREC == PREC_FP32) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int qt = 0; qt < QT; ++qt)
                    acc[rt][qt] = __builtin_amdgcn_mfma_f32_32x32x2f32(x[rt][0][j], q[qt][0][j], acc[rt][qt], 0, 0, 0);
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

template <int PREC, int METRIC, int QT, int RT, int PX, int PQ, int KP, int CAP, int WPS>
__global__ void __launch_bounds__(256, WPS)
scan_topk_kernel(const float* __restrict__ X, const float* __restrict__ rowscale, const uint32_t* __restrict__ mask,
                 const float* __restrict__ Qt, int G, int64_t N, int B, int64_t n_steps, int steps_per_wg,
                 float* __restrict__ cand_s, uint32_t* __restrict__ cand_i, uint32_t* __restrict__ gthr,
                 uint32_t* __restrict__ gslots) {
    static_assert(PX % PQ == 0, "query prefetch depth must divide the corpus prefetch depth");
    static_assert(PQ <= QG_EXTRA, "query prefetch deeper than the duplicated groups");
    constexpr int QB = 32 * QT;
    constexpr int SR = 4 * RT * 32;  // rows per step
    __shared__ float s_sc[QB * CAP];
    __shared__ uint32_t s_ix[QB * CAP];
    __shared__ int s_cnt[QB];
    __shared__ float s_thr[QB];
    __shared__ uint32_t s_best[QB];  // order key of the best score appended so far
    __shared__ uint32_t s_pub[QB];   // ... and of the last one published
    __shared__ float s_rs[2][SR];  // row scales, double-buffered by step parity

    const int lane = threadIdx.x & 63;
    // wave index made provably uniform: every tile/group address below is then
    // scalar (SGPR base) + lane*16 (one VGPR), keeping VGPRs for the pipeline.
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int n_wg = gridDim.x;
    const int wg = blockIdx.x;
    const int qb = blockIdx.y;
    const int lane4 = lane * 4;

    for (int i = threadIdx.x; i < QB; i += 256) {
        s_cnt[i] = 0;
        s_best[i] = 0;
        s_pub[i] = 0;
        s_thr[i] = -INFINITY;
    }

    const int64_t s_begin = (int64_t)wg * steps_per_wg;
    const int64_t s_end = s_begin + steps_per_wg < n_steps ? s_begin + steps_per_wg : n_steps;
    // super-tile addressing: group g of row tile t starts at blk(t, g); consecutive
    // groups are GBLK blocks apart (fp32: 4 sub tiles; split: 2 planes x 4 sub
    // tiles), sub tiles of one group adjacent, the lo plane 4 blocks after hi.
    constexpr int NPL = PREC + 1;
    constexpr int GBLK = 4 * NPL;
    constexpr size_t GSTEP = GBLK * BLOCK_FLOATS;
    constexpr size_t PLANE = 4 * BLOCK_FLOATS;
    auto blk = [](uint64_t t, int g, int GG) -> size_t {
        return (((size_t)(t >> 2) * GG + g) * GBLK + (t & 3)) * BLOCK_FLOATS;
    };
    // the query tiles carry QG_EXTRA duplicated leading groups after group G-1, so
    // the query stream of a step runs through groups PQ .. G+PQ-1 without a wrap
    const float* Qbase = Qt + blk((uint64_t)(qb * QT), 0, G + QG_EXTRA);

    f32x4 xr[PX][RT][NPL], qr[PQ][QT][NPL];
    if (s_begin < s_end) {
        const float* xs = X + blk((uint64_t)((s_begin * 4 + wv) * RT), 0, G);
#pragma unroll
        for (int p = 0; p < PX; ++p)
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int pl = 0; pl < NPL; ++pl)
                    xr[p][rt][pl] = *(const f32x4*)(xs + p * GSTEP + pl * PLANE + rt * BLOCK_FLOATS + lane4);
#pragma unroll
        for (int p = 0; p < PQ; ++p)
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                for (int pl = 0; pl < NPL; ++pl)
                    qr[p][qt][pl] = *(const f32x4*)(Qbase + p * GSTEP + pl * PLANE + qt * BLOCK_FLOATS + lane4);
    }

    // row scales of the first step; later steps' are loaded one step ahead (next
    // to the shared-threshold load) so that no step starts with a load whose
    // value is needed at once (that wait would drain the corpus prefetch)
    static_assert(SR % 256 == 0, "row scales are staged SR/256 per thread");
    constexpr int RSN = SR / 256;
    if (s_begin < s_end)
        for (int i = 0; i < RSN; ++i) s_rs[s_begin & 1][threadIdx.x + 256 * i] = rowscale[s_begin * SR + threadIdx.x + 256 * i];
#ifdef VDB_STAMP
    unsigned long long st_k = 0, st_e = 0, st_e0 = 0, st_t0 = STAMP_NOW();
    unsigned long long st_bar = 0, st_sc = 0, st_ins = 0, st_rt = 0, st_rounds = 0, st_compacts = 0;
    unsigned long long st_pub_start = 0, st_pub = 0;
#endif
    for (int64_t s = s_begin; s < s_end; ++s) {
#ifdef VDB_STAMP
        const unsigned long long st_a = STAMP_NOW();
#endif
        // row scales of this step -> LDS, read in the epilogue after the K-loop's
        // barrier; buffer s&1 was last read in step s-2's epilogue (before step
        // s-1's barriers)
        const float* rs_buf = s_rs[s & 1];

        const int64_t t0 = (s * 4 + wv) * RT;
        const float* xs = X + blk((uint64_t)t0, 0, G);
        const float* xn = (s + 1 < s_end) ? X + blk((uint64_t)(t0 + 4 * RT), 0, G) : xs;
        f32x16 acc[RT][QT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                for (int v = 0; v < 16; ++v) acc[rt][qt][v] = 0.0f;

        // One group: 4 k-steps of MFMAs on slot p, then refill slot p with the group
        // PX ahead (from this step, or the next step's first groups).  The refill is
        // pinned right after the MFMAs; left to itself the scheduler sinks it and
        // shortens the prefetch distance.
        auto group = [&](const int p, const float* xsrc, const float* qsrc) {
            const int pq = p % PQ;
            group_mfma<PREC, RT, QT>(xr[p], qr[pq], acc);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int pl = 0; pl < NPL; ++pl)
                    xr[p][rt][pl] = *(const f32x4*)(xsrc + pl * PLANE + rt * BLOCK_FLOATS + lane4);
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                for (int pl = 0; pl < NPL; ++pl)
                    qr[pq][qt][pl] = *(const f32x4*)(qsrc + pl * PLANE + qt * BLOCK_FLOATS + lane4);
            __builtin_amdgcn_sched_barrier(0);
        };
        int gb = 0;
        for (; gb < G - PX; gb += PX) {
#pragma unroll
            for (int p = 0; p < PX; ++p)
                group(p, xs + (size_t)(gb + p + PX) * GSTEP, Qbase + (size_t)(gb + p + PQ) * GSTEP);
        }
        // shared thresholds (max over workgroups of their KP-th best so far), read
        // before the last PX groups so the load hides under them; any value read,
        // however stale (even an L1 copy), is a valid lower bound
        uint32_t gk[QT];
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
            const int qg = qb * QB + qt * 32 + (lane & 31);
            gk[qt] = qg < B ? gthr[qg] : 0u;
        }
        float rsn[RSN];
        const int64_t sn = s + 1 < s_end ? s + 1 : s;
#pragma unroll
        for (int i = 0; i < RSN; ++i) rsn[i] = rowscale[sn * SR + threadIdx.x + 256 * i];
#pragma unroll
        for (int p = 0; p < PX; ++p) group(p, xn + (size_t)p * GSTEP, Qbase + (size_t)(gb + p + PQ) * GSTEP);
#ifdef VDB_STAMP
        const unsigned long long st_b = STAMP_NOW();
        st_k += st_b - st_a;
#endif
        __syncthreads();  // s_rs visible
#pragma unroll
        for (int i = 0; i < RSN; ++i) s_rs[(s + 1) & 1][threadIdx.x + 256 * i] = rsn[i];
#ifdef VDB_STAMP
        const unsigned long long st_b2 = STAMP_NOW();
        st_bar += st_b2 - st_b;
#endif

        // ---- epilogue -----------------------------------------------------------
        // Scores replace the accumulators in place; pass bits are built branch-free;
        // the LDS append runs only for score slots where some lane of the wave
        // passes (after the first steps that is almost never), so the common step
        // costs ~2 VALU per score.  A full buffer leaves a score pending, to be
        // re-tested after the buffer is compacted (retry loop below).
        uint32_t pend[RT][QT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            const int64_t t = t0 + rt;
            const uint32_t mword = mask ? mask[t] : 0xFFFFFFFFu;
            const float* rsp = rs_buf + (wv * RT + rt) * 32 + 4 * (lane >> 5);
            f32x4 rs4[4];
#pragma unroll
            for (int m = 0; m < 4; ++m) rs4[m] = *(const f32x4*)(rsp + 8 * m);
            uint32_t okbits = 0;
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                const int ro = (v & 3) + 8 * (v >> 2) + 4 * (lane >> 5);
                okbits |= (((mword >> ro) & 1u) && (t * 32 + ro < N)) ? (1u << v) : 0u;
            }
#pragma unroll
            for (int qt = 0; qt < QT; ++qt) {
                const int ql = qt * 32 + (lane & 31);
                const float thr = fmaxf(s_thr[ql], key_to_float(gk[qt]));
                uint32_t pm = 0;
#pragma unroll
                for (int v = 0; v < 16; ++v) {
                    const float a = acc[rt][qt][v];
                    const float rs = rs4[v >> 2][v & 3];
                    const float sc = METRIC == 0 ? a * rs : fmaf(2.0f, a, -rs);
                    acc[rt][qt][v] = sc;
                    pm |= sc > thr ? (1u << v) : 0u;
                }
                pend[rt][qt] = (qb * QB + ql < B) ? (pm & okbits) : 0u;
            }
        }
#ifdef VDB_STAMP
        const unsigned long long st_b3 = STAMP_NOW();
        st_sc += st_b3 - st_b2;
#endif
        // one LDS atomic per lane reserves slots for all of its passing scores of
        // the tile; slots past CAP leave the score pending
        auto insert_tile = [&](int rt, int qt) -> uint32_t {
            const uint32_t pm = pend[rt][qt];
            if (!__any(pm != 0)) return 0u;
            const int ql = qt * 32 + (lane & 31);
            const int base = pm ? atomicAdd(&s_cnt[ql], __popc(pm)) : 0;
            float mx = -INFINITY;
#pragma unroll
            for (int v = 0; v < 16; ++v) mx = ((pm >> v) & 1u) ? fmaxf(mx, acc[rt][qt][v]) : mx;
            if (pm) atomicMax(&s_best[ql], order_key(mx));
            uint32_t left = 0;
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                if ((pm >> v) & 1u) {
                    const int pos = base + __popc(pm & ((1u << v) - 1u));
                    if (pos < CAP) {
                        const int ro = (v & 3) + 8 * (v >> 2) + 4 * (lane >> 5);
                        s_sc[ql * CAP + pos] = acc[rt][qt][v];
                        s_ix[ql * CAP + pos] = (uint32_t)((t0 + rt) * 32 + ro);
                    } else {
                        left |= 1u << v;
                    }
                }
            }
            return left;
        };
        uint32_t any_left = 0;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int qt = 0; qt < QT; ++qt) {
                pend[rt][qt] = insert_tile(rt, qt);
                any_left |= pend[rt][qt];
            }
#ifdef VDB_STAMP
        const unsigned long long st_b4 = STAMP_NOW();
        st_ins += st_b4 - st_b3;
#endif
        while (__syncthreads_or(any_left != 0)) {
#ifdef VDB_STAMP
            ++st_rounds;
#endif
            for (int q = wv; q < QB; q += 4)
                if (s_cnt[q] >= CAP) {
#ifdef VDB_STAMP
                    ++st_compacts;
#endif
                    compact_query<KP, CAP>(s_sc + q * CAP, s_ix + q * CAP, s_cnt + q, s_thr + q,
                                           qb * QB + q < B ? gthr + qb * QB + q : nullptr);
                }
            __syncthreads();
            any_left = 0;
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
                for (int qt = 0; qt < QT; ++qt) {
                    const float thr = fmaxf(s_thr[qt * 32 + (lane & 31)], key_to_float(gk[qt]));
                    uint32_t keep = 0;
#pragma unroll
                    for (int v = 0; v < 16; ++v) keep |= acc[rt][qt][v] > thr ? (1u << v) : 0u;
                    pend[rt][qt] &= keep;
                    pend[rt][qt] = insert_tile(rt, qt);
                    any_left |= pend[rt][qt];
                }
            }
        }
#ifdef VDB_STAMP
        const unsigned long long st_b5 = STAMP_NOW();
        st_pub_start = st_b5;
#endif
        // ---- publish: slot (query, wg % KP) of gslots holds the max over a fixed set
        // of workgroups of their best score, so the KP slots of a query are scores of
        // KP distinct rows and their minimum is a lower bound of the global KP-th best
        // (DESIGN.md §3.2).  Only queries whose best improved are republished.
        // Published after this workgroup's steps 1, 2, 4, 8, ... (each costs a global
        // round trip, and the bound moves little once every slot is filled).
        const int64_t sd = s - s_begin + 1;
        if ((sd & (sd - 1)) == 0 || s + 1 == s_end) {
            constexpr int QPW = QB / 4;
            bool improved = false;
            uint32_t best = 0;
            int qg = 0;
            if (lane < QPW) {
                const int q = wv + 4 * lane;
                qg = qb * QB + q;
                best = s_best[q];
                improved = qg < B && best > s_pub[q];
                if (improved) {
                    s_pub[q] = best;
                    atomicMax(gslots + (size_t)qg * KP + (wg % KP), best);
                }
            }
            if (__any(improved) && improved) {
                // all KP slot loads in flight at once (one round trip)
                const uint32_t* sl = gslots + (size_t)qg * KP;
                uint32_t mn = 0xFFFFFFFFu;
#pragma unroll
                for (int j = 0; j < KP; j += 4) {
                    const uint4 v4 = *(const uint4*)(sl + j);
                    mn = min(min(mn, min(v4.x, v4.y)), min(v4.z, v4.w));
                }
                atomicMax(gthr + qg, mn);
            }
        }
#ifdef VDB_STAMP
        const unsigned long long st_c = STAMP_NOW();
        st_pub += st_c - st_pub_start;
        st_rt += st_pub_start - st_b4;
        st_e += st_c - st_b;
        if (s == s_begin) st_e0 = st_c - st_b;
#endif
    }
#ifdef VDB_STAMP
    if (lane == 0 && blockIdx.y == 0) {
        const int w = wg * 4 + wv;
        g_scan_stamps[w][0] = st_k;
        g_scan_stamps[w][1] = st_e;
        g_scan_stamps[w][2] = st_pub;
        g_scan_stamps[w][3] = STAMP_NOW() - st_t0;
        g_scan_stamps[w][4] = st_bar;
        g_scan_stamps[w][5] = st_sc;
        g_scan_stamps[w][6] = st_ins;
        g_scan_stamps[w][7] = st_rt;
    }
#endif

    // ---- flush: sorted top-KP of every query of the block ------------------------
    __syncthreads();
    for (int q = wv; q < QB; q += 4) {
        const int qg = qb * QB + q;
        const size_t base = ((size_t)(qg < B ? qg : 0) * n_wg + wg) * KP;
        flush_query<KP, CAP>(s_sc + q * CAP, s_ix + q * CAP, s_cnt + q, s_thr + q, qg < B ? cand_s + base : nullptr,
                             cand_i + base);
    }
}

template <int PREC, int METRIC, int QT, int RT, int PX, int PQ, int KP, int CAP, int WPS>
static hipError_t scan_dispatch(const float* X, const float* rowscale, const uint32_t* mask, const float* Qt, int G,
                                int64_t N, int B, int n_qblocks, int64_t n_steps, int n_wg, int spw, float* cs,
                                uint32_t* ci, uint32_t* gthr, uint32_t* gslots, hipStream_t st) {
    hipLaunchKernelGGL((scan_topk_kernel<PREC, METRIC, QT, RT, PX, PQ, KP, CAP, WPS>), dim3(n_wg, n_qblocks), dim3(256),
                       0, st, X, rowscale, mask, Qt, G, N, B, n_steps, spw, cs, ci, gthr, gslots);
    return hipGetLastError();
}

// Variants (RT row tiles of 32 per wave, corpus PX groups ahead, queries PQ ahead):
//   fp32  0: RT=2 PX=4 PQ=4, 2 waves/SIMD     1: RT=4 PX=4 PQ=2, 2 waves/SIMD
//         2: RT=4 PX=8 PQ=2, 1 wave/SIMD (accumulators in AGPRs)
//   bf16x3 0: RT=2 PX=4 PQ=2, 1 wave/SIMD     1: RT=4 PX=4 PQ=2, 1 wave/SIMD
//         2: RT=2 PX=8 PQ=2, 1 wave/SIMD
static int variant_rt(int prec, int variant) {
    if (prec == PREC_FP32) return variant == 0 ? 2 : 4;
    return variant == 1 ? 4 : 2;
}
static int variant_px(int prec, int variant) {
    if (prec == PREC_FP32) return variant == 2 ? 8 : 4;
    return variant == 2 ? 8 : 4;
}

int scan_rows_per_step(int prec, int variant) { return 4 * 32 * variant_rt(prec, variant); }

bool scan_variant_ok(int prec, int variant, int G) {
    return variant >= 0 && variant <= 2 && G % variant_px(prec, variant) == 0;
}

hipError_t launch_scan_topk(int prec, int metric, int KP, int variant, const float* X, const float* rowscale,
                            const uint32_t* mask, const float* Qt, int G, int64_t N, int B, int n_qblocks,
                            int64_t n_steps, int n_wg, int spw, float* cs, uint32_t* ci, uint32_t* gthr,
                            uint32_t* gslots, hipStream_t st) {
    if (!scan_variant_ok(prec, variant, G)) return hipErrorInvalidValue;
#define VDB_SCAN(P, M, QT, KPV, V, RT, PX, PQ, W)                                                               \
    if (prec == P && metric == M && KP == KPV && variant == V)                                                 \
        return scan_dispatch<P, M, QT, RT, PX, PQ, KPV, (KPV == 32 ? 4 : 2) * KPV, W>(                          \
            X, rowscale, mask, Qt, G, N, B, n_qblocks, n_steps, n_wg, spw, cs, ci, gthr, gslots, st);
#define VDB_SCAN_ALL(M)                                                                                        \
    VDB_SCAN(0, M, 2, 32, 0, 2, 4, 4, 2) VDB_SCAN(0, M, 2, 64, 0, 2, 4, 4, 2)                                  \
    VDB_SCAN(0, M, 2, 128, 0, 2, 4, 4, 1) VDB_SCAN(0, M, 1, 256, 0, 2, 4, 4, 1)                                \
    VDB_SCAN(0, M, 2, 32, 1, 4, 4, 2, 2) VDB_SCAN(0, M, 2, 64, 1, 4, 4, 2, 2)                                  \
    VDB_SCAN(0, M, 2, 32, 2, 4, 8, 2, 1) VDB_SCAN(0, M, 2, 64, 2, 4, 8, 2, 1)                                  \
    VDB_SCAN(1, M, 2, 32, 0, 2, 4, 2, 1) VDB_SCAN(1, M, 2, 64, 0, 2, 4, 2, 1)                                  \
    VDB_SCAN(1, M, 2, 128, 0, 2, 4, 2, 1) VDB_SCAN(1, M, 1, 256, 0, 2, 4, 2, 1)                                \
    VDB_SCAN(1, M, 2, 32, 1, 4, 4, 2, 1) VDB_SCAN(1, M, 2, 64, 1, 4, 4, 2, 1)                                  \
    VDB_SCAN(1, M, 2, 128, 1, 4, 4, 2, 1)                                                                      \
    VDB_SCAN(1, M, 2, 32, 2, 2, 8, 2, 1) VDB_SCAN(1, M, 2, 64, 2, 2, 8, 2, 1)
    VDB_SCAN_ALL(0)
    VDB_SCAN_ALL(1)
#undef VDB_SCAN_ALL
#undef VDB_SCAN
    return hipErrorInvalidValue;
}

}  // namespace vdb

#ifdef VDB_STAMP
extern "C" int vdb_debug_scan_stamps(unsigned long long* out, int n_waves) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(vdb::g_scan_stamps), (size_t)n_waves * 8 * sizeof(unsigned long long));
}
#endif
