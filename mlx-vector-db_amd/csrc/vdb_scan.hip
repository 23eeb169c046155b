// vdb_scan.hip — gfx950 kernels of the brute-force distance + top-k path.
//
// Pipeline for one search:
//   prep_queries -> pilot_scores + pilot_bound (seed the shared bound from sampled tiles)
//   -> scan_topk (MFMA candidate pass, fp32 or bf16x3, fused per-WG top-KP, appended
//      to global per-query candidate lists)
//   -> finish (vdb_exact.hip: select top-KP, exact fp64 rerank, top-k, certificate)
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
#include "vdb_scan_common.h"

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
// Top-KP per query lives in LDS: an append buffer of CAP >= 2 KP entries
// (score, row) per query (larger CAP = fewer compaction rounds while the first
// steps fill it) plus a threshold (the KP-th best after the last compaction).  A
// score enters only if it beats the threshold; when a buffer fills, one wave
// selects the best KP by bisection (compact_query).  Invariant used by the certificate in
// rerank: every row not in the final list scored <= the list's KP-th entry.

// Epilogue scoring of one step: scores replace the accumulators (cosine a * inv|x|,
// L2 2a - |x|^2) and pend[rt][qt] gets the bits of the scores above the query's
// threshold.  The common case costs ~1.5 VALU per score: scale + max3, then one
// compare per tile; the per-score bits (and the row mask / N checks) are built
// only for tiles where some lane of the wave passes.
template <int METRIC, int RT, int QT>
__device__ __forceinline__ void score_tiles(f32x16 (&acc)[RT][QT], const f32x4 (&rs4)[RT][4], const float (&thr)[QT],
                                            const uint32_t (&mword)[RT], const bool (&qok)[QT], int64_t t0, int64_t N,
                                            uint32_t (&pend)[RT][QT]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
            float mx = -INFINITY;
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                const float a = acc[rt][qt][v];
                const float rs = rs4[rt][v >> 2][v & 3];
                const float sc = METRIC == 0 ? a * rs : fmaf(2.0f, a, -rs);
                acc[rt][qt][v] = sc;
                mx = fmaxf(mx, sc);
            }
            pend[rt][qt] = 0u;
            if (__any(qok[qt] && mx > thr[qt])) {
                const int64_t t = t0 + rt;
                uint32_t pm = 0;
#pragma unroll
                for (int v = 0; v < 16; ++v) {
                    const int ro = (v & 3) + 8 * (v >> 2) + 4 * (lane >> 5);
                    const bool ok = ((mword[rt] >> ro) & 1u) && (t * 32 + ro < N);
                    pm |= (ok && acc[rt][qt][v] > thr[qt]) ? (1u << v) : 0u;
                }
                pend[rt][qt] = qok[qt] ? pm : 0u;
            }
        }
    }
}

template <int PREC, int METRIC, int QT, int RT, int PX, int PQ, int KP, int CAP, int PUB, int WPS, bool NT, int NW,
          bool FLAGSYNC>
__global__ void __launch_bounds__(64 * NW, WPS)
scan_topk_kernel(const float* __restrict__ X, const float* __restrict__ rowscale, const uint32_t* __restrict__ mask,
                 const float* __restrict__ Qt, int G, int64_t N, int B, int64_t n_steps, int steps_per_wg,
                 int n_qb, int n_wg_all, float* __restrict__ gl_s, uint32_t* __restrict__ gl_i,
                 uint32_t* __restrict__ gl_cnt, int64_t gl_cap, uint32_t* __restrict__ gthr,
                 uint32_t* __restrict__ gslots) {
    static_assert(PX % PQ == 0, "query prefetch depth must divide the corpus prefetch depth");
    static_assert(PQ <= QG_EXTRA, "query prefetch deeper than the duplicated groups");
    constexpr int QB = 32 * QT;
    __shared__ float s_sc[QB * CAP];
    __shared__ uint32_t s_ix[QB * CAP];
    __shared__ int s_cnt[QB];
    __shared__ float s_thr[QB];
    __shared__ uint32_t s_best[NW][QB];  // per wave: order key of the best score appended so far (PUB)
    __shared__ uint32_t s_pub[NW][QB];   // ... and of the last one published
    __shared__ uint32_t s_sh[QB];    // shared bound from the slots (order key), this WG's view
    __shared__ int s_need;           // some wave holds scores that did not fit: compaction round wanted
    __shared__ int s_done;           // waves past their last step

    const int lane = threadIdx.x & 63;
    if (FLAGSYNC && threadIdx.x == 0) {
        s_need = 0;
        s_done = 0;
    }
    // wave index made provably uniform: every tile/group address below is then
    // scalar (SGPR base) + lane*16 (one VGPR), keeping VGPRs for the pipeline.
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // XCD-aware placement (1-D grid): workgroups are dealt round-robin over the 8
    // XCDs, so the n_qb query blocks of one row range get block ids with the same
    // residue mod 8 and adjacent dispatch slots: they stream the same corpus rows
    // together through one XCD's L2 instead of each pulling them from HBM.
    int wg, qb;
    xcd_map(n_qb, wg, qb);
    const int n_wg = n_wg_all;
    const int lane4 = lane * 4;

    for (int i = threadIdx.x; i < QB; i += 64 * NW) {
        s_cnt[i] = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            s_best[w][i] = 0;
            s_pub[w][i] = 0;
        }
        s_sh[i] = 0;
        s_thr[i] = -INFINITY;
    }
    __syncthreads();
    // slot publishing: lane group pq_i (LPQ lanes) of wave wv serves query pq = wv + NW pq_i
    constexpr int QPW = QB / NW;
    constexpr int LPQ = 64 / QPW;
    constexpr int SL = KP / LPQ;
    constexpr int SLV = SL / 4 > 0 ? SL / 4 : 1;
    static_assert(!PUB || SL % 4 == 0, "slots per lane must be whole uint4 loads");
    static_assert(LPQ >= NW, "a lane group publishes one best per wave");
    const int pq_r = lane % LPQ;
    const int pq = wv + NW * (lane / LPQ);
    const int pqg = qb * QB + pq;
    uint4 sv[SLV];
    bool sv_pending = false;

    const int64_t s_begin = (int64_t)wg * steps_per_wg;
    const int64_t s_end = s_begin + steps_per_wg < n_steps ? s_begin + steps_per_wg : n_steps;
    // super-tile addressing: group g of row tile t starts at blk(t, g); consecutive
    // groups are GBLK blocks apart (fp32: 4 sub tiles; split: 2 planes x 4 sub
    // tiles), sub tiles of one group adjacent, the lo plane 4 blocks after hi.
    constexpr int XPL = Planes<PREC>::XPL, QPL = Planes<PREC>::QPL;
    constexpr int GBLK = 4 * Planes<PREC>::LPL;
    constexpr size_t GSTEP = GBLK * BLOCK_FLOATS;
    constexpr size_t PLANE = 4 * BLOCK_FLOATS;
    auto blk = [](uint64_t t, int g, int GG) -> size_t {
        return (((size_t)(t >> 2) * GG + g) * GBLK + (t & 3)) * BLOCK_FLOATS;
    };
    // the query tiles carry QG_EXTRA duplicated leading groups after group G-1, so
    // the query stream of a step runs through groups PQ .. G+PQ-1 without a wrap
    const float* Qbase = Qt + blk((uint64_t)(qb * QT), 0, G + QG_EXTRA);

    f32x4 xr[PX][RT][XPL], qr[PQ][QT][QPL];
    if (s_begin < s_end) {
        const float* xs = X + blk((uint64_t)((s_begin * NW + wv) * RT), 0, G);
#pragma unroll
        for (int p = 0; p < PX; ++p)
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int pl = 0; pl < XPL; ++pl)
                    xr[p][rt][pl] = corpus_ld<NT>(xs + p * GSTEP + pl * PLANE + rt * BLOCK_FLOATS + lane4);
#pragma unroll
        for (int p = 0; p < PQ; ++p)
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                for (int pl = 0; pl < QPL; ++pl)
                    qr[p][qt][pl] = *(const f32x4*)(Qbase + p * GSTEP + pl * PLANE + qt * BLOCK_FLOATS + lane4);
    }
    // epilogue inputs of step s (see the step loop)
    auto load_epi = [&](int64_t st_, uint32_t (&g_)[QT], f32x4 (&r_)[RT][4], uint32_t (&m_)[RT]) {
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
            const int qg = qb * QB + qt * 32 + (lane & 31);
            g_[qt] = qg < B ? gthr[qg] : 0u;
        }
        const int64_t tt = (st_ * NW + wv) * RT;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            const float* rsp = rowscale + (tt + rt) * 32 + 4 * (lane >> 5);
#pragma unroll
            for (int m = 0; m < 4; ++m) r_[rt][m] = *(const f32x4*)(rsp + 8 * m);
            // the caller's bitmap holds ceil(N/32) words (vdb.h): tiles past it are rows >= N
            m_[rt] = !mask ? 0xFFFFFFFFu : (tt + rt < ((N + 31) >> 5) ? mask[tt + rt] : 0u);
        }
    };
    uint32_t gkn[QT];
    f32x4 rsn[RT][4];
    uint32_t mwn[RT];
    if (s_begin < s_end) load_epi(s_begin, gkn, rsn, mwn);
#ifdef VDB_STAMP
    unsigned long long st_k = 0, st_e = 0, st_e0 = 0, st_t0 = STAMP_NOW();
    unsigned long long st_bar = 0, st_sc = 0, st_ins = 0, st_rt = 0, st_rounds = 0, st_compacts = 0;
    unsigned long long st_pub_start = 0, st_pub = 0;
#endif
    for (int64_t s = s_begin; s < s_end; ++s) {
#ifdef VDB_STAMP
        const unsigned long long st_a = STAMP_NOW();
#endif
        const int64_t t0 = (s * NW + wv) * RT;
        const float* xs = X + blk((uint64_t)t0, 0, G);
        const float* xn = (s + 1 < s_end) ? X + blk((uint64_t)(t0 + NW * RT), 0, G) : xs;
        f32x16 acc[RT][QT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                for (int v = 0; v < 16; ++v) acc[rt][qt][v] = 0.0f;

        // One group: the MFMAs of slot p, then refill slot p with the group PX ahead
        // (from this step, or the next step's first groups).  The refill is pinned
        // right after the MFMAs; left to itself the scheduler sinks it and shortens
        // the prefetch distance.
        auto group = [&](const int p, const float* xsrc, const float* qsrc) {
            const int pq = p % PQ;
            group_mfma<PREC, RT, QT>(xr[p], qr[pq], acc);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int pl = 0; pl < XPL; ++pl)
                    xr[p][rt][pl] = corpus_ld<NT>(xsrc + pl * PLANE + rt * BLOCK_FLOATS + lane4);
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                for (int pl = 0; pl < QPL; ++pl)
                    qr[pq][qt][pl] = *(const f32x4*)(qsrc + pl * PLANE + qt * BLOCK_FLOATS + lane4);
            __builtin_amdgcn_sched_barrier(0);
        };
        int gb = 0;
        for (; gb < G - PX; gb += PX) {
#pragma unroll
            for (int p = 0; p < PX; ++p)
                group(p, xs + (size_t)(gb + p + PX) * GSTEP, Qbase + (size_t)(gb + p + PQ) * GSTEP);
        }
        // The epilogue's global inputs (shared thresholds -- any value read, however
        // stale, even an L1 copy, is a valid lower bound --, the row scales of this
        // wave's rows: lane l needs rows (v & 3) + 8 (v >> 2) + 4 (l >> 5) of each
        // tile, and the tile masks) are loaded one step ahead, before the last PX
        // groups: waiting for them never drains the corpus stream, and their latency
        // is covered even when a step is only a few groups long (small D).
        uint32_t gk[QT];
        f32x4 rs4[RT][4];
        uint32_t mword[RT];
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) gk[qt] = gkn[qt];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            mword[rt] = mwn[rt];
#pragma unroll
            for (int m = 0; m < 4; ++m) rs4[rt][m] = rsn[rt][m];
        }
        if (s + 1 < s_end) load_epi(s + 1, gkn, rsn, mwn);
#pragma unroll
        for (int p = 0; p < PX; ++p) group(p, xn + (size_t)p * GSTEP, Qbase + (size_t)(gb + p + PQ) * GSTEP);
#ifdef VDB_STAMP
        const unsigned long long st_b = STAMP_NOW();
        st_k += st_b - st_a;
        const unsigned long long st_b2 = st_b;
#endif

        // ---- epilogue -----------------------------------------------------------
        // Scores replace the accumulators in place; pass bits are built branch-free;
        // the LDS append runs only for score slots where some lane of the wave
        // passes (after the first steps that is almost never), so the common step
        // costs ~2 VALU per score.  A full buffer leaves a score pending, to be
        // re-tested after the buffer is compacted (retry loop below).
        uint32_t pend[RT][QT];
        {
            float thr[QT];
            bool qok[QT];
#pragma unroll
            for (int qt = 0; qt < QT; ++qt) {
                const int ql = qt * 32 + (lane & 31);
                thr[qt] = fmaxf(s_thr[ql], key_to_float(PUB ? max(gk[qt], s_sh[ql]) : gk[qt]));
#ifdef VDB_STAMP
                // diagnostic bounds (stamp build only, wrong results): PUB 2 = no insertion
                // after the first step, PUB 3 = no insertion at all
                if ((PUB == 2 && s > s_begin) || PUB == 3) thr[qt] = INFINITY;
#endif
                qok[qt] = qb * QB + ql < B;
            }
            score_tiles<METRIC, RT, QT>(acc, rs4, thr, mword, qok, t0, N, pend);
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
            if constexpr (PUB) {
                float mx = -INFINITY;
#pragma unroll
                for (int v = 0; v < 16; ++v) mx = ((pm >> v) & 1u) ? fmaxf(mx, acc[rt][qt][v]) : mx;
                if (pm) atomicMax(&s_best[wv][ql], order_key(mx));
            }
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
        // Compaction rounds without a per-step barrier: a wave left with scores that
        // did not fit raises s_need and waits at B1; every other wave looks at s_need
        // at the end of each of its steps (and once more after its last one, below)
        // and joins.  In the common step (nothing left anywhere) no wave waits for
        // another, so the four corpus streams of a workgroup never realign.  The flag
        // is looked at once per step: after a round a wave stays only while it still
        // holds leftovers (else waves past their last step, which raise the flag every
        // round, would keep it here forever).
        // Without FLAGSYNC (measured better for long steps) every step
        // ends in one workgroup barrier instead, which doubles as B1.
        for (bool joined = false;; joined = true) {
            if constexpr (!FLAGSYNC) {
                if (!__syncthreads_or(any_left != 0)) break;
            } else {
                const bool mine = __any(any_left != 0);
                if (mine && lane == 0) lds_flag_st(&s_need, 1);
                if (!mine && (joined || !__builtin_amdgcn_readfirstlane(lds_flag_ld(&s_need)))) break;
                __syncthreads();  // B1: all waves here, each with leftovers or having seen the flag
            }
#ifdef VDB_STAMP
            ++st_rounds;
#endif
            for (int q = wv; q < QB; q += NW)
                if (s_cnt[q] >= CAP) {
#ifdef VDB_STAMP
                    ++st_compacts;
#endif
                    compact_query<KP, CAP>(s_sc + q * CAP, s_ix + q * CAP, s_cnt + q, s_thr + q,
                                           qb * QB + q < B ? gthr + qb * QB + q : nullptr);
                }
            if (FLAGSYNC && threadIdx.x == 0) lds_flag_st(&s_need, 0);  // nobody reads it between B1 and B2
            __syncthreads();  // B2
            any_left = 0;
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
                for (int qt = 0; qt < QT; ++qt) {
                    const int ql = qt * 32 + (lane & 31);
                    const float thr = fmaxf(s_thr[ql], key_to_float(PUB ? max(gk[qt], s_sh[ql]) : gk[qt]));
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
        if constexpr (PUB) {
            // ---- publish: slot (query, (NW wg + w) % KP) of gslots holds the max over a
            // fixed set of waves (disjoint rows) of their best score, so the KP slots of a
            // query are scores of KP distinct rows and their minimum is a lower bound of
            // the global KP-th best; NW slots per workgroup so that KP
            // slots fill even when there are fewer than KP workgroups.  A group of LPQ lanes serves one query: its leader
            // publishes (no-return atomic), all of them load SL slots each.  The slot
            // loads are consumed one step later (min over the group's lanes -> gthr and
            // s_sh): by then the next step's corpus loads, which are younger, have been
            // waited for, so reading the slots never drains the HBM stream.
            if (sv_pending) {
                uint32_t mn = 0xFFFFFFFFu;
#pragma unroll
                for (int j = 0; j < SLV; ++j) mn = min(min(mn, min(sv[j].x, sv[j].y)), min(sv[j].z, sv[j].w));
#pragma unroll
                for (int off = 1; off < LPQ; off <<= 1) mn = min(mn, (uint32_t)__shfl_xor((int)mn, off, 64));
                if (pq_r == 0 && pqg < B) {
                    atomicMax(gthr + pqg, mn);
                    atomicMax(&s_sh[pq], mn);
                }
                sv_pending = false;
            }
            const int64_t sd = s - s_begin + 1;
            if ((sd & (sd - 1)) == 0 || s + 1 == s_end) {
                int improved = 0;
                if (pq_r < NW && pqg < B) {  // lane r of the group publishes wave r's best
                    const uint32_t best = s_best[pq_r][pq];
                    improved = best > s_pub[pq_r][pq];
                    if (improved) {
                        s_pub[pq_r][pq] = best;
                        atomicMax(gslots + (size_t)pqg * KP_MAX + ((wg * NW + pq_r) % KP), best);
                    }
                }
#pragma unroll
                for (int off = 1; off < LPQ; off <<= 1) improved |= __shfl_xor(improved, off, 64);
                if (improved) {
                    const uint32_t* sl = gslots + (size_t)pqg * KP_MAX + pq_r * SL;
#pragma unroll
                    for (int j = 0; j < SLV; ++j) sv[j] = *(const uint4*)(sl + 4 * j);
                }
                sv_pending = improved;
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
        const int w = wg * NW + wv;
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

    // Past the last step: keep answering compaction rounds (B1 / B2 as in the step
    // loop) until every wave of the workgroup is here; a wave still stepping sees
    // s_need (raised by this wave every round) at its next step end.  All waves
    // read s_done == NW after the same B1, so they leave together.
    if (FLAGSYNC && lane == 0) atomicAdd(&s_done, 1);
    for (; FLAGSYNC;) {
        if (lane == 0) lds_flag_st(&s_need, 1);
        __syncthreads();  // B1
        if (__builtin_amdgcn_readfirstlane(lds_flag_ld(&s_done)) == NW) break;
        for (int q = wv; q < QB; q += NW)
            if (s_cnt[q] >= CAP)
                compact_query<KP, CAP>(s_sc + q * CAP, s_ix + q * CAP, s_cnt + q, s_thr + q,
                                       qb * QB + q < B ? gthr + qb * QB + q : nullptr);
        if (threadIdx.x == 0) lds_flag_st(&s_need, 0);
        __syncthreads();  // B2
    }

    // ---- flush: entries above the shared bound -> global per-query lists ----------
    // (wave wv flushes queries wv + NW i; lane i holds query i's bound)
    __syncthreads();
    (void)n_wg;
    uint32_t tkey = 0;
    if (lane < QPW && qb * QB + wv + NW * lane < B) tkey = max(gthr[qb * QB + wv + NW * lane], PUB ? s_sh[wv + NW * lane] : 0u);
    if constexpr (PUB) {
        if (sv_pending) {  // a slot read-back still in flight: fold it in
            uint32_t mn = 0xFFFFFFFFu;
#pragma unroll
            for (int j = 0; j < SLV; ++j) mn = min(min(mn, min(sv[j].x, sv[j].y)), min(sv[j].z, sv[j].w));
#pragma unroll
            for (int off = 1; off < LPQ; off <<= 1) mn = min(mn, (uint32_t)__shfl_xor((int)mn, off, 64));
            if (pq_r == 0 && pqg < B) atomicMax(gthr + pqg, mn);
        }
    }
    append_flush<CAP>(s_sc, s_ix, s_cnt, wv, NW, QPW, qb * QB, B, tkey, gl_s, gl_i, gl_cnt, gl_cap);
}

// =============================================================================
// Candidate pass, wave-private variant (KP <= 32, 64 queries per block)
// =============================================================================
// Same K-loop as scan_topk_kernel, but every wave keeps its own top-KP per query
// (LDS append buffer of CAPW entries per query and wave), so the step loop has no
// workgroup barrier: a wave's epilogue never stalls the other three waves' corpus
// streams.  Shared bounds as before (gthr: compaction thresholds + the deferred
// slot minimum; s_sh: this workgroup's view of the slot minimum).  At the end each
// wave appends the entries above the shared bound T to a global per-query list
// (one returning atomic per query per wave); select_topk then takes the top KP of
// each list.  Certificate invariant: every row not in a list scored <= max(the
// list's KP-th entry, final gthr).
template <int PREC, int METRIC, int QT, int RT, int PX, int PQ, int KP, int CAPW>
__global__ void __launch_bounds__(256, 1)
scan_topk_priv_kernel(const float* __restrict__ X, const float* __restrict__ rowscale,
                      const uint32_t* __restrict__ mask, const float* __restrict__ Qt, int G, int64_t N, int B,
                      int64_t n_steps, int steps_per_wg, int n_qb, int n_wg_all, float* __restrict__ gl_s,
                      uint32_t* __restrict__ gl_i,
                      uint32_t* __restrict__ gl_cnt, int64_t gl_cap, uint32_t* __restrict__ gthr,
                      uint32_t* __restrict__ gslots) {
    static_assert(PX % PQ == 0, "query prefetch depth must divide the corpus prefetch depth");
    static_assert(PQ <= QG_EXTRA, "query prefetch deeper than the duplicated groups");
    constexpr int QB = 32 * QT;
    static_assert(QB <= 64 && KP % 4 == 0 && CAPW % 64 == 0, "one lane per query; whole uint4 slot loads");
    __shared__ float s_sc[4][QB * CAPW];
    __shared__ uint32_t s_ix[4][QB * CAPW];
    __shared__ int s_cnt[4][QB];
    __shared__ float s_thr[4][QB];
    __shared__ uint32_t s_best[4][QB];
    __shared__ uint32_t s_sh[QB];

    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int wg, qb;
    xcd_map(n_qb, wg, qb);
    (void)n_wg_all;
    const int lane4 = lane * 4;
    float* bs = s_sc[wv];
    uint32_t* bi = s_ix[wv];
    int* bc = s_cnt[wv];
    float* bt = s_thr[wv];
    uint32_t* bb = s_best[wv];
    if (lane < QB) {
        bc[lane] = 0;
        bt[lane] = -INFINITY;
        bb[lane] = 0;
        if (wv == 0) s_sh[lane] = 0;
    }
    __syncthreads();

    const int64_t s_begin = (int64_t)wg * steps_per_wg;
    const int64_t s_end = s_begin + steps_per_wg < n_steps ? s_begin + steps_per_wg : n_steps;
    constexpr int XPL = Planes<PREC>::XPL, QPL = Planes<PREC>::QPL;
    constexpr int GBLK = 4 * Planes<PREC>::LPL;
    constexpr size_t GSTEP = GBLK * BLOCK_FLOATS;
    constexpr size_t PLANE = 4 * BLOCK_FLOATS;
    auto blk = [](uint64_t t, int g, int GG) -> size_t {
        return (((size_t)(t >> 2) * GG + g) * GBLK + (t & 3)) * BLOCK_FLOATS;
    };
    const float* Qbase = Qt + blk((uint64_t)(qb * QT), 0, G + QG_EXTRA);
    // slot publishing: lane q < QB serves query q of the block
    const int pqg = qb * QB + lane;
    const bool pq_ok = lane < QB && pqg < B;
    const int slot = (wg * 4 + wv) % KP;
    uint32_t pub = 0;  // this wave's last published best (order key)
    uint4 sv[KP / 4];
    bool sv_pending = false;

    f32x4 xr[PX][RT][XPL], qr[PQ][QT][QPL];
    if (s_begin < s_end) {
        const float* xs = X + blk((uint64_t)((s_begin * 4 + wv) * RT), 0, G);
#pragma unroll
        for (int p = 0; p < PX; ++p)
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int pl = 0; pl < XPL; ++pl)
                    xr[p][rt][pl] = corpus_ld<false>(xs + p * GSTEP + pl * PLANE + rt * BLOCK_FLOATS + lane4);
#pragma unroll
        for (int p = 0; p < PQ; ++p)
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                for (int pl = 0; pl < QPL; ++pl)
                    qr[p][qt][pl] = *(const f32x4*)(Qbase + p * GSTEP + pl * PLANE + qt * BLOCK_FLOATS + lane4);
    }
    // epilogue inputs of step s (see the step loop)
    auto load_epi = [&](int64_t st_, uint32_t (&g_)[QT], f32x4 (&r_)[RT][4], uint32_t (&m_)[RT]) {
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
            const int qg = qb * QB + qt * 32 + (lane & 31);
            g_[qt] = qg < B ? gthr[qg] : 0u;
        }
        const int64_t tt = (st_ * 4 + wv) * RT;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            const float* rsp = rowscale + (tt + rt) * 32 + 4 * (lane >> 5);
#pragma unroll
            for (int m = 0; m < 4; ++m) r_[rt][m] = *(const f32x4*)(rsp + 8 * m);
            // the caller's bitmap holds ceil(N/32) words (vdb.h): tiles past it are rows >= N
            m_[rt] = !mask ? 0xFFFFFFFFu : (tt + rt < ((N + 31) >> 5) ? mask[tt + rt] : 0u);
        }
    };
    uint32_t gkn[QT];
    f32x4 rsn[RT][4];
    uint32_t mwn[RT];
    if (s_begin < s_end) load_epi(s_begin, gkn, rsn, mwn);
    uint32_t gk[QT];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) gk[qt] = 0;

    for (int64_t s = s_begin; s < s_end; ++s) {
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
        auto group = [&](const int p, const float* xsrc, const float* qsrc) {
            const int pq = p % PQ;
            group_mfma<PREC, RT, QT>(xr[p], qr[pq], acc);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int pl = 0; pl < XPL; ++pl)
                    xr[p][rt][pl] = corpus_ld<false>(xsrc + pl * PLANE + rt * BLOCK_FLOATS + lane4);
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                for (int pl = 0; pl < QPL; ++pl)
                    qr[pq][qt][pl] = *(const f32x4*)(qsrc + pl * PLANE + qt * BLOCK_FLOATS + lane4);
            __builtin_amdgcn_sched_barrier(0);
        };
        int gb = 0;
        for (; gb < G - PX; gb += PX) {
#pragma unroll
            for (int p = 0; p < PX; ++p)
                group(p, xs + (size_t)(gb + p + PX) * GSTEP, Qbase + (size_t)(gb + p + PQ) * GSTEP);
        }
        // epilogue inputs: this step's (loaded a step ahead), then the next step's
        // (see scan_topk_kernel)
        f32x4 rs4[RT][4];
        uint32_t mword[RT];
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) gk[qt] = gkn[qt];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            mword[rt] = mwn[rt];
#pragma unroll
            for (int m = 0; m < 4; ++m) rs4[rt][m] = rsn[rt][m];
        }
        if (s + 1 < s_end) load_epi(s + 1, gkn, rsn, mwn);
#pragma unroll
        for (int p = 0; p < PX; ++p) group(p, xn + (size_t)p * GSTEP, Qbase + (size_t)(gb + p + PQ) * GSTEP);

        // ---- epilogue (wave-local) ----------------------------------------------
        uint32_t pend[RT][QT];
        {
            float thr[QT];
            bool qok[QT];
#pragma unroll
            for (int qt = 0; qt < QT; ++qt) {
                const int ql = qt * 32 + (lane & 31);
                thr[qt] = fmaxf(bt[ql], key_to_float(max(gk[qt], s_sh[ql])));
                qok[qt] = qb * QB + ql < B;
            }
            score_tiles<METRIC, RT, QT>(acc, rs4, thr, mword, qok, t0, N, pend);
        }
        auto insert_tile = [&](int rt, int qt) -> uint32_t {
            const uint32_t pm = pend[rt][qt];
            if (!__any(pm != 0)) return 0u;
            const int ql = qt * 32 + (lane & 31);
            const int base = pm ? atomicAdd(&bc[ql], __popc(pm)) : 0;
            float mx = -INFINITY;
#pragma unroll
            for (int v = 0; v < 16; ++v) mx = ((pm >> v) & 1u) ? fmaxf(mx, acc[rt][qt][v]) : mx;
            if (pm) atomicMax(&bb[ql], order_key(mx));
            uint32_t left = 0;
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                if ((pm >> v) & 1u) {
                    const int pos = base + __popc(pm & ((1u << v) - 1u));
                    if (pos < CAPW) {
                        const int ro = (v & 3) + 8 * (v >> 2) + 4 * (lane >> 5);
                        bs[ql * CAPW + pos] = acc[rt][qt][v];
                        bi[ql * CAPW + pos] = (uint32_t)((t0 + rt) * 32 + ro);
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
        while (__any(any_left != 0)) {
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
            unsigned long long full = __ballot(lane < QB && bc[lane < QB ? lane : 0] >= CAPW);
            while (full) {
                const int q = __builtin_ctzll(full);
                full &= full - 1;
                compact_query<KP, CAPW>(bs + q * CAPW, bi + q * CAPW, bc + q, bt + q,
                                        qb * QB + q < B ? gthr + qb * QB + q : nullptr);
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
            any_left = 0;
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
                for (int qt = 0; qt < QT; ++qt) {
                    const int ql = qt * 32 + (lane & 31);
                    const float thr = fmaxf(bt[ql], key_to_float(max(gk[qt], s_sh[ql])));
                    uint32_t keep = 0;
#pragma unroll
                    for (int v = 0; v < 16; ++v) keep |= acc[rt][qt][v] > thr ? (1u << v) : 0u;
                    pend[rt][qt] &= keep;
                    pend[rt][qt] = insert_tile(rt, qt);
                    any_left |= pend[rt][qt];
                }
            }
        }
        // ---- publish (lane q = query q; the slot read-back is consumed one step later) --
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        if (sv_pending) {
            uint32_t mn = 0xFFFFFFFFu;
#pragma unroll
            for (int j = 0; j < KP / 4; ++j) mn = min(min(mn, min(sv[j].x, sv[j].y)), min(sv[j].z, sv[j].w));
            atomicMax(gthr + pqg, mn);
            atomicMax(&s_sh[lane], mn);
            sv_pending = false;
        }
        const int64_t sd = s - s_begin + 1;
        if ((sd & (sd - 1)) == 0 || s + 1 == s_end) {
            const uint32_t best = pq_ok ? bb[lane] : 0u;
            if (pq_ok && best > pub) {
                pub = best;
                atomicMax(gslots + (size_t)pqg * KP_MAX + slot, best);
                const uint32_t* sl = gslots + (size_t)pqg * KP_MAX;
#pragma unroll
                for (int j = 0; j < KP / 4; ++j) sv[j] = *(const uint4*)(sl + 4 * j);
                sv_pending = true;
            }
        }
    }

    // ---- flush: entries above the shared bound -> global per-query lists ----------
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    uint32_t tkey = pq_ok ? max(gthr[pqg], s_sh[lane]) : 0u;
    if (sv_pending) {
        uint32_t mn = 0xFFFFFFFFu;
#pragma unroll
        for (int j = 0; j < KP / 4; ++j) mn = min(min(mn, min(sv[j].x, sv[j].y)), min(sv[j].z, sv[j].w));
        atomicMax(gthr + pqg, mn);
        tkey = max(tkey, mn);
    }
    append_flush<CAPW>(bs, bi, bc, 0, 1, QB, qb * QB, B, tkey, gl_s, gl_i, gl_cnt, gl_cap);
}

// Top KP (sorted by score desc, row asc; sentinel padded) of each query's global
// append list.  One wave per query: <= 256 entries in registers (bitonic), more
// through the LDS streaming top-k (only when the shared bound was weak).
constexpr int SELECT_REG = 256;
__global__ void __launch_bounds__(64) select_topk_kernel(const float* __restrict__ gl_s, const uint32_t* __restrict__ gl_i,
                                                         const uint32_t* __restrict__ gl_cnt, int64_t gl_cap, int KP,
                                                         float* __restrict__ out_s, uint32_t* __restrict__ out_i) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x;
    const int q = blockIdx.x;
    const int64_t c = min((int64_t)gl_cnt[q], gl_cap);
    const float* ls = gl_s + (size_t)q * gl_cap;
    const uint32_t* li = gl_i + (size_t)q * gl_cap;
    float* os = out_s + (size_t)q * KP;
    uint32_t* oi = out_i + (size_t)q * KP;
    if (c <= SELECT_REG) {
        constexpr int E = SELECT_REG / 64;
        float v[E];
        uint32_t x[E];
#pragma unroll
        for (int i = 0; i < E; ++i) {
            const int e = i * 64 + lane;
            v[i] = e < c ? ls[e] : -INFINITY;
            x[i] = e < c ? li[e] : 0xFFFFFFFFu;
        }
        wave_sort_desc<float, uint32_t, E>(v, x);
#pragma unroll
        for (int i = 0; i < E; ++i) {
            const int e = i * 64 + lane;
            if (e < KP) {
                os[e] = v[i];
                oi[e] = x[i];
            }
        }
        for (int e = SELECT_REG + lane; e < KP; e += 64) {
            os[e] = -INFINITY;
            oi[e] = 0xFFFFFFFFu;
        }
        return;
    }
    WaveTopK<float, uint32_t> tk;
    tk.init(reinterpret_cast<float*>(smem),
            reinterpret_cast<uint32_t*>(smem + (size_t)WaveTopK<float, uint32_t>::capacity(KP) * sizeof(float)), KP);
    for (int64_t f0 = 0; f0 < c; f0 += 64) {
        const int64_t f = f0 + lane;
        const bool in = f < c;
        tk.offer(in, in ? ls[f] : -INFINITY, in ? li[f] : 0xFFFFFFFFu);
    }
    tk.finish();
    for (int e = lane; e < KP; e += 64) {
        os[e] = tk.bk[e];
        oi[e] = tk.bi[e];
    }
}

hipError_t launch_select_topk(const float* gl_s, const uint32_t* gl_i, const uint32_t* gl_cnt, int64_t gl_cap, int KP,
                              int B, float* out_s, uint32_t* out_i, hipStream_t st) {
    const size_t lds = (size_t)WaveTopK<float, uint32_t>::capacity(KP) * 8;
    hipLaunchKernelGGL(select_topk_kernel, dim3(B), dim3(64), lds, st, gl_s, gl_i, gl_cnt, gl_cap, KP, out_s, out_i);
    return hipGetLastError();
}

template <int PREC, int METRIC, int QT, int RT, int PX, int PQ, int KP, int CAPW>
static hipError_t scan_priv_dispatch(const float* X, const float* rowscale, const uint32_t* mask, const float* Qt,
                                     int G, int64_t N, int B, int n_qblocks, int64_t n_steps, int n_wg, int spw,
                                     float* gl_s, uint32_t* gl_i, uint32_t* gl_cnt, int64_t gl_cap, uint32_t* gthr,
                                     uint32_t* gslots, hipStream_t st) {
    const int n_wg8 = (n_wg + 7) / 8 * 8;
    hipLaunchKernelGGL((scan_topk_priv_kernel<PREC, METRIC, QT, RT, PX, PQ, KP, CAPW>), dim3(n_wg8 * n_qblocks),
                       dim3(256), 0, st, X, rowscale, mask, Qt, G, N, B, n_steps, spw, n_qblocks, n_wg8, gl_s, gl_i,
                       gl_cnt, gl_cap, gthr, gslots);
    return hipGetLastError();
}

// wave-private candidate pass: fp32 variant 0 (measured faster there), bf16x3 variant 1
bool scan_priv(int prec, int variant, int KP) { return KP == 32 && prec == PREC_FP32 && variant == 0; }

int scan_priv_capw() { return 64; }

hipError_t launch_scan_topk_priv(int prec, int metric, int KP, const float* X, const float* rowscale,
                                 const uint32_t* mask, const float* Qt, int G, int64_t N, int B, int n_qblocks,
                                 int64_t n_steps, int n_wg, int spw, float* gl_s, uint32_t* gl_i, uint32_t* gl_cnt,
                                 int64_t gl_cap, uint32_t* gthr, uint32_t* gslots, hipStream_t st) {
    if (KP != 32 || G % 4 != 0) return hipErrorInvalidValue;
#define VDB_PRIV(P, M, PQV)                                                                                   \
    if (prec == P && metric == M)                                                                             \
        return scan_priv_dispatch<P, M, 2, 2, 4, PQV, 32, 64>(X, rowscale, mask, Qt, G, N, B, n_qblocks, n_steps, \
                                                            n_wg, spw, gl_s, gl_i, gl_cnt, gl_cap, gthr, gslots, st);
    VDB_PRIV(0, 0, 4) VDB_PRIV(0, 1, 4)
#undef VDB_PRIV
    return hipErrorInvalidValue;
}

// =============================================================================
// Pilot bound: scores of a strided sample of row tiles, KP-th best per query
// =============================================================================
// A cold scan inserts almost every score of its first steps (no bound yet), which
// costs more than the rest of the epilogue.  The pilot scores n_sample evenly
// spaced row tiles with exactly the scan's arithmetic (same group order through
// group_mfma, same row scale), so its KP-th best per query is the KP-th best of a
// subset of the rows the scan will score identically: a valid lower bound of the
// global KP-th best, written to gthr before the scan starts.
template <int PREC, int METRIC, int QT>
__global__ void __launch_bounds__(64) pilot_scores_kernel(const float* __restrict__ X, const float* __restrict__ rowscale,
                                                          const uint32_t* __restrict__ mask, const float* __restrict__ Qt,
                                                          int G, int64_t N, int B, int64_t n_tiles, int n_sample,
                                                          uint32_t* __restrict__ pslots) {
    constexpr int QB = 32 * QT;
    constexpr int XPL = Planes<PREC>::XPL, QPL = Planes<PREC>::QPL;
    constexpr int GBLK = 4 * Planes<PREC>::LPL;
    constexpr size_t GSTEP = GBLK * BLOCK_FLOATS;
    constexpr size_t PLANE = 4 * BLOCK_FLOATS;
    auto blk = [](uint64_t t, int g, int GG) -> size_t {
        return (((size_t)(t >> 2) * GG + g) * GBLK + (t & 3)) * BLOCK_FLOATS;
    };
    const int lane = threadIdx.x;
    const int i = blockIdx.x;
    const int qb = blockIdx.y;
    const uint64_t t = (uint64_t)((int64_t)i * n_tiles / n_sample);
    const float* xs = X + blk(t, 0, G) + lane * 4;
    const float* qs = Qt + blk((uint64_t)(qb * QT), 0, G + QG_EXTRA) + lane * 4;
    f32x16 acc[1][QT];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[0][qt][v] = 0.0f;
    // one wave, groups in the scan's order (bit-identical accumulators), loads PP
    // groups ahead so the tile costs a few HBM round trips, not G of them
    constexpr int PP = 12;
    f32x4 xr[PP][1][XPL], qr[PP][QT][QPL];
    auto load = [&](int slot, int g) {
        if (g < G) {
#pragma unroll
            for (int pl = 0; pl < XPL; ++pl) xr[slot][0][pl] = *(const f32x4*)(xs + g * GSTEP + pl * PLANE);
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                for (int pl = 0; pl < QPL; ++pl)
                    qr[slot][qt][pl] = *(const f32x4*)(qs + g * GSTEP + pl * PLANE + qt * BLOCK_FLOATS);
        }
    };
#pragma unroll
    for (int p = 0; p < PP; ++p) load(p, p);
    for (int g0 = 0; g0 < G; g0 += PP) {
#pragma unroll
        for (int p = 0; p < PP; ++p) {
            if (g0 + p < G) {
                group_mfma<PREC, 1, QT>(xr[p], qr[p], acc);
                load(p, g0 + p + PP);
            }
        }
    }
    // the tile's best eligible score per query -> pilot slot (i mod PILOT_SLOTS): the
    // slots hold scores of distinct rows, so the KP-th largest slot is a lower bound
    // of the global KP-th best (pilot_bound_kernel)
    const uint32_t mword = mask ? mask[t] : 0xFFFFFFFFu;
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
        const int q = qb * QB + qt * 32 + (lane & 31);
        float best = -INFINITY;
#pragma unroll
        for (int v = 0; v < 16; ++v) {
            const int ro = (v & 3) + 8 * (v >> 2) + 4 * (lane >> 5);
            const float rs = rowscale[t * 32 + ro];
            const float a = acc[0][qt][v];
            const float sc = METRIC == 0 ? a * rs : fmaf(2.0f, a, -rs);
            const bool ok = ((mword >> ro) & 1u) && ((int64_t)t * 32 + ro < N);
            best = ok ? fmaxf(best, sc) : best;
        }
        best = fmaxf(best, __shfl_xor(best, 32, 64));  // the tile's two row halves (lane, lane + 32)
        if (lane < 32 && q < B && best != -INFINITY) atomicMax(pslots + pslot_at(q, i % PILOT_SLOTS, B), order_key(best));
    }
}

// gthr[q] = max(gthr[q], KP-th largest pilot slot) when at least KP slots are
// filled: one wave per query, ballot bisection over the 256 slots (4 per lane).
__global__ void __launch_bounds__(64) pilot_bound_kernel(const uint32_t* __restrict__ pslots, int B, int KP,
                                                         uint32_t* __restrict__ gthr) {
    const int q = blockIdx.x;
    const int lane = threadIdx.x;
    constexpr int E = PILOT_SLOTS / 64;
    uint32_t v[E];
#pragma unroll
    for (int i = 0; i < E; ++i) v[i] = pslots[pslot_at(q, i * 64 + lane, B)];
    int filled = 0;
#pragma unroll
    for (int i = 0; i < E; ++i) filled += __popcll(__ballot(v[i] != 0u));
    if (filled < KP) return;
    uint32_t T = 0;
    for (int bit = 31; bit >= 0; --bit) {
        const uint32_t c = T | (1u << bit);
        int n = 0;
#pragma unroll
        for (int i = 0; i < E; ++i) n += __popcll(__ballot(v[i] >= c));
        if (n >= KP) T = c;
    }
    if (lane == 0 && T != 0) atomicMax(gthr + q, T);
}

hipError_t launch_pilot(int prec, int metric, int KP, const float* X, const float* rowscale, const uint32_t* mask,
                        const float* Qt, int G, int64_t N, int B, int n_qblocks, int QB, int n_sample,
                        uint32_t* pslots, uint32_t* gthr, hipStream_t st) {
    const int64_t n_tiles = (N + 31) / 32;
    if (n_sample > n_tiles) n_sample = (int)n_tiles;
    if (n_sample <= 0 || KP > PILOT_SLOTS) return hipSuccess;
    const dim3 grid(n_sample, n_qblocks);
    bool launched = false;
#define VDB_PILOT(P, M, QTV)                                                                                     \
    if (!launched && prec == P && metric == M && QB == 32 * QTV) {                                               \
        hipLaunchKernelGGL((pilot_scores_kernel<P, M, QTV>), grid, dim3(64), 0, st, X, rowscale, mask, Qt, G, N,   \
                           B, n_tiles, n_sample, pslots);                                                        \
        launched = true;                                                                                         \
    }
    VDB_PILOT(0, 0, 2) VDB_PILOT(0, 1, 2) VDB_PILOT(0, 0, 1) VDB_PILOT(0, 1, 1)
#undef VDB_PILOT
    if (!launched) return hipErrorInvalidValue;
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_pilot_bound(pslots, B, KP, gthr, st);
}

hipError_t launch_pilot_bound(uint32_t* pslots, int B, int KP, uint32_t* gthr, hipStream_t st) {
    hipLaunchKernelGGL(pilot_bound_kernel, dim3(B), dim3(64), 0, st, pslots, B, KP, gthr);
    return hipGetLastError();
}

template <int V, int PREC, int METRIC, int QT, int RT, int PX, int PQ, int KP, int CAP, int PUB, int WPS, bool NT, int NW>
static hipError_t scan_dispatch(const float* X, const float* rowscale, const uint32_t* mask, const float* Qt, int G,
                                int64_t N, int B, int n_qblocks, int64_t n_steps, int n_wg, int spw, float* gl_s,
                                uint32_t* gl_i, uint32_t* gl_cnt, int64_t gl_cap, uint32_t* gthr, uint32_t* gslots,
                                int lockstep, hipStream_t st) {
    const int n_wg8 = (n_wg + 7) / 8 * 8;
    // flag-gated step ends are built for the default variants only (others run lockstep)
    if constexpr (V == 0) {
        if (!lockstep) {
            hipLaunchKernelGGL((scan_topk_kernel<PREC, METRIC, QT, RT, PX, PQ, KP, CAP, PUB, WPS, NT, NW, true>),
                               dim3(n_wg8 * n_qblocks), dim3(64 * NW), 0, st, X, rowscale, mask, Qt, G, N, B, n_steps,
                               spw, n_qblocks, n_wg8, gl_s, gl_i, gl_cnt, gl_cap, gthr, gslots);
            return hipGetLastError();
        }
    }
    hipLaunchKernelGGL((scan_topk_kernel<PREC, METRIC, QT, RT, PX, PQ, KP, CAP, PUB, WPS, NT, NW, false>),
                       dim3(n_wg8 * n_qblocks), dim3(64 * NW), 0, st, X, rowscale, mask, Qt, G, N, B, n_steps, spw,
                       n_qblocks, n_wg8, gl_s, gl_i, gl_cnt, gl_cap, gthr, gslots);
    return hipGetLastError();
}

// Variants of this (fp32) candidate pass (RT row tiles of 32 per wave, corpus PX groups
// ahead, queries PQ ahead, CAP append-buffer entries per query, PUB = slot publishing):
//   0: RT=2 PX=4 PQ=4, 2 waves/SIMD    1: RT=4 PX=4 PQ=2    2: RT=4 PX=8 PQ=2, 1 wave/SIMD
// The split-bf16 passes are vdb_scan2.hip.
static int variant_rt(int, int variant) { return variant == 0 ? 2 : 4; }
static int variant_px(int, int variant) { return variant == 2 ? 8 : 4; }

int scan_wgs_per_cu(int, int, int) { return 1; }

int scan_rows_per_step(int prec, int variant) { return 4 * 32 * variant_rt(prec, variant); }

bool scan_variant_ok(int prec, int variant, int G) {
    return prec == PREC_FP32 && variant >= 0 && variant <= 2 && G % variant_px(prec, variant) == 0;
}

hipError_t launch_scan_topk(int prec, int metric, int KP, int variant, const float* X, const float* rowscale,
                            const uint32_t* mask, const float* Qt, int G, int64_t N, int B, int n_qblocks,
                            int64_t n_steps, int n_wg, int spw, float* gl_s, uint32_t* gl_i, uint32_t* gl_cnt,
                            int64_t gl_cap, uint32_t* gthr, uint32_t* gslots, int lockstep, hipStream_t st) {
    if (!scan_variant_ok(prec, variant, G)) return hipErrorInvalidValue;
#define VDB_SCAN_NT(P, M, QT, KPV, V, RT, PX, PQ, CAPV, PUB, W, NT)                                           \
    if (prec == P && metric == M && KP == KPV && variant == V && (n_qblocks == 1) == NT)                       \
        return scan_dispatch<V, P, M, QT, RT, PX, PQ, KPV, CAPV, PUB, W, NT, 4>(X, rowscale, mask, Qt, G, N, B,      \
                                                                        n_qblocks, n_steps, n_wg, spw, gl_s, gl_i, \
                                                                        gl_cnt, gl_cap, gthr, gslots, lockstep, st);
// VDB_SCAN: default load policy only; VDB_SCAN2: plus the non-temporal build for one query block
#define VDB_SCAN(P, M, QT, KPV, V, RT, PX, PQ, CAPV, PUB, W)                                                     \
    if (prec == P && metric == M && KP == KPV && variant == V)                                                 \
        return scan_dispatch<V, P, M, QT, RT, PX, PQ, KPV, CAPV, PUB, W, false, 4>(X, rowscale, mask, Qt, G, N, B,   \
                                                                           n_qblocks, n_steps, n_wg, spw, gl_s,    \
                                                                           gl_i, gl_cnt, gl_cap, gthr, gslots, lockstep, st);
#define VDB_SCAN2(P, M, QT, KPV, V, RT, PX, PQ, CAPV, PUB, W)                                                    \
    VDB_SCAN_NT(P, M, QT, KPV, V, RT, PX, PQ, CAPV, PUB, W, true)                                              \
    VDB_SCAN_NT(P, M, QT, KPV, V, RT, PX, PQ, CAPV, PUB, W, false)
#define VDB_SCAN_ALL(M)                                                                                        \
    VDB_SCAN2(0, M, 2, 32, 0, 2, 4, 4, 128, 1, 2) VDB_SCAN2(0, M, 2, 64, 0, 2, 4, 4, 128, 1, 2)                \
    VDB_SCAN(0, M, 2, 128, 0, 2, 4, 4, 256, 1, 1) VDB_SCAN(0, M, 1, 256, 0, 2, 4, 4, 512, 1, 1)                \
    VDB_SCAN(0, M, 2, 32, 1, 4, 4, 2, 128, 1, 2) VDB_SCAN(0, M, 2, 64, 1, 4, 4, 2, 128, 1, 2)                  \
    VDB_SCAN(0, M, 2, 32, 2, 4, 8, 2, 128, 1, 1) VDB_SCAN(0, M, 2, 64, 2, 4, 8, 2, 128, 1, 1)
    VDB_SCAN_ALL(0)
    VDB_SCAN_ALL(1)
#undef VDB_SCAN_ALL
#undef VDB_SCAN2
#undef VDB_SCAN_NT
#undef VDB_SCAN
    return hipErrorInvalidValue;
}

}  // namespace vdb

#ifdef VDB_STAMP
extern "C" int vdb_debug_scan_stamps(unsigned long long* out, int n_waves) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(vdb::g_scan_stamps), (size_t)n_waves * 8 * sizeof(unsigned long long));
}
#endif
