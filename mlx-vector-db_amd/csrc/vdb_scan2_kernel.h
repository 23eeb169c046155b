// vdb_scan2_kernel.h — the split-bf16 candidate pass kernel template and its launch
// templates (included by vdb_scan2.hip and by the per-(precision, metric) instantiation
// units vdb_scan2_{b3,b1}{c,l}.hip, which the build compiles in parallel).
// MFMA scores of a 64-query block against the whole corpus fused with a per-workgroup
// top-KP, appended to global per-query candidate lists (pipeline: vdb_scan.hip header).
//
// Shape, from the K-loop ablation (profiles/scripts/scan_micro2.hip, MI355X, C2 1M x 768):
//   * 4 waves, one per SIMD; each wave owns RT = 4 row tiles (128 rows) x 2 query tiles per
//     step: per 16-dim group 4 corpus blocks per plane (HBM, default or nt policy) and
//     2 x 2 query blocks (L2) feed 24 (bf16x3) or 16 (bf16) v_mfma_f32_32x32x16_bf16, so
//     the query operand costs half the bytes of the corpus operand (RT = 2: twice as many):
//     bf16x3 K-loop 515 -> 480 us (6.25 -> 6.7 TB/s), bf16 hi plane 308 -> 252 us.
//   * the corpus loads run PX groups ahead in registers (bf16x3 PX = 2, bf16 PX = 4: equal
//     bytes in flight); for small D (C4: D = 128) the query block sits in LDS instead
//     (QLDS), which takes the query loads off the vector-memory path (TA) that the corpus
//     stream of C4's 8 query blocks already saturates.
//   * no row scale in the epilogue: for cosine the split copy holds the NORMALISED rows
//     (x / |x| rounded to fp32, then split; the query is normalised too), so the
//     accumulator IS the score; for L2 the accumulator starts at -|x|^2 / 2 (rinit), so it
//     ends at q.x - |x|^2 / 2 = score / 2.  The start value is written by one fp32 MFMA per
//     tile (A = the rows' rinit in column 0, B = ones in row 0: exact), so a lane holds one
//     rinit value per tile instead of the 16 its accumulator rows need.  Per 16-score tile the common case is 16
//     accumulator reads, 8 max3 and one compare; the pass bits, row validity (mask / N)
//     and the LDS insert run only for tiles where some lane passes.
// Invariant for the certificate (vdb_exact.hip finish_kernel): every row not in the final
// list scored (this arithmetic) <= max(its workgroup's KP-th best, the final shared bound).
#pragma once
#include "vdb_common.h"
#include "vdb_internal.h"
#include "vdb_scan_common.h"

#include <atomic>

namespace vdb {

#ifdef VDB_STAMP
// Diagnostic build only (make stamp): per-wave phase cycles of scan2_kernel:
// [0] prologue, [1] k-loop, [2] epilogue (insert + compaction rounds), [3] total,
// [4] (unused), [5] flush, [6] steps, [7] start time (absolute)
static __device__ unsigned long long g_scan2_stamps[1 << 16][8];
#define S2_NOW() __builtin_amdgcn_s_memtime()
#endif

#ifndef VDB_S2_RT
#define VDB_S2_RT 4
#endif
#ifndef VDB_S2_NW
#define VDB_S2_NW 4
#endif
// the step's group loop: one loop with the tail selected inside (1) or the tail peeled (0)
#ifndef VDB_S2_ONELOOP
#define VDB_S2_ONELOOP 0
#endif
constexpr int S2_RT = VDB_S2_RT;  // row tiles (32 rows) per wave per step
constexpr int S2_NW = VDB_S2_NW;  // waves per workgroup
constexpr int S2_ROWS = S2_RT * S2_NW * 32;

// row-valid bits of row tile t for this lane: bit v <-> row 32 t + (v & 3) + 8 (v >> 2) + 4 (lane >> 5)
__device__ __forceinline__ uint32_t tile_valid16(const uint32_t* mask, int64_t t, int64_t N, int lane) {
    uint32_t w = 0xFFFFFFFFu;
    if (mask) w = t < ((N + 31) >> 5) ? mask[t] : 0u;
    const int64_t rem = N - t * 32;
    if (rem < 32) w &= rem <= 0 ? 0u : ((1u << rem) - 1u);
    w >>= 4 * (lane >> 5);
    return (w & 0xFu) | ((w >> 4) & 0xF0u) | ((w >> 8) & 0xF00u) | ((w >> 12) & 0xF000u);
}

// IEEE-754 2019 maximum (NaN-propagating, no input canonicalisation): a chain of gfx950
// v_maximum3_f32, 8 instructions per 16 scores instead of 16 canonicalising v_max_f32 +
// 8 v_max3_f32 under IEEE mode (the scores are never NaN: non-finite rows are rejected
// at ingest, queries on the host / by the caller's contract)
#ifdef VDB_S2_IEEE_MAX  // A/B build: IEEE fmaxf (canonicalising) tile maxima
#define S2_MAXIMUM(a, b) fmaxf(a, b)
#else
#define S2_MAXIMUM(a, b) __builtin_elementwise_maximum(a, b)
#endif
__device__ __forceinline__ float tile_max16(const f32x16& a) {  // a depth-3 tree of 3-input maxima
#define S2_MAX3(x, y, z) S2_MAXIMUM(S2_MAXIMUM(x, y), z)
    const float m0 = S2_MAX3(a[0], a[1], a[2]), m1 = S2_MAX3(a[3], a[4], a[5]), m2 = S2_MAX3(a[6], a[7], a[8]);
    const float m3 = S2_MAX3(a[9], a[10], a[11]), m4 = S2_MAX3(a[12], a[13], a[14]);
    return S2_MAXIMUM(S2_MAX3(m0, m1, m2), S2_MAX3(m3, m4, a[15]));
#undef S2_MAX3
}

// split-layout block of (row tile t, 16-dim group g) with GG groups: [t/4][GG][2 planes][4][1 KiB]
__device__ __forceinline__ size_t s2_blk(uint64_t t, int g, int GG) {
    return (((size_t)(t >> 2) * GG + g) * 8 + (t & 3)) * BLOCK_FLOATS;
}

// The pilot bound of one query (one wave): the rank-th largest of its PILOT_SLOTS pilot slots
// (vdb_api.cpp pilot_rank), 0 when fewer slots are filled.  Small ranks by repeated wave
// maxima (remove one copy of the maximum per round), larger ones by ballot bisection.
constexpr int PILOT_E = PILOT_SLOTS / 64;  // slots per lane

__device__ __forceinline__ uint32_t pilot_slot_rank(uint32_t (&v)[PILOT_E], int rank) {
    constexpr int E = PILOT_E;
    const int lane = threadIdx.x & 63;
    int filled = 0;
#pragma unroll
    for (int i = 0; i < E; ++i) filled += __popcll(__ballot(v[i] != 0u));
    if (filled < rank) return 0u;
    if (rank <= 16) {
        for (int r = 1;; ++r) {
            uint32_t m = v[0];
#pragma unroll
            for (int i = 1; i < E; ++i) m = max(m, v[i]);
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, off, 64));
            if (r == rank) return m;
            // drop one copy of m: the lowest lane holding it, its first register
            int hit = -1;
#pragma unroll
            for (int i = E - 1; i >= 0; --i) hit = v[i] == m ? i : hit;
            const unsigned long long who = __ballot(hit >= 0);
            if (lane == __ffsll((long long)who) - 1) {
#pragma unroll
                for (int i = 0; i < E; ++i)
                    if (i == hit) v[i] = 0u;
            }
        }
    }
    uint32_t T = 0;
    for (int bit = 31; bit >= 0; --bit) {
        const uint32_t c = T | (1u << bit);
        int n = 0;
#pragma unroll
        for (int i = 0; i < E; ++i) n += __popcll(__ballot(v[i] >= c));
        if (n >= rank) T = c;
    }
    return T;
}

// GC > 0: the dimension groups as a compile-time constant (short rows, C4: 8), so the group
// loop unrolls; the runtime loop made the register allocator copy 4 of the 8 accumulator
// tiles between register sets on every step (256 v_accvgpr_mov per step at C4).
// RT row tiles per wave (the default S2_RT = 4; the 128-query shape QT = 4 takes 2, so the
// accumulators stay at 128 registers).  KW < KP: a workgroup keeps only its KW best per query
// (smaller LDS buffers, which the 128-query blocks need); its compactions then do not raise
// gthr (a workgroup's KW-th best is no bound of the global KP-th) and at its end it raises gthr
// to its drop bound (its KW-th best), which keeps the certificate's invariant (rows outside the
// lists score <= max(a_KP, final gthr)); the finish then certifies as usual.
template <int PREC, int METRIC, int QT, int PX, int KP, int CAP, bool NT, bool QLDS, bool FLAGSYNC, int GC = 0,
          int RT_ = S2_RT, int KW = KP>
__global__ void __launch_bounds__(64 * S2_NW, 1)
scan2_kernel(const float* __restrict__ Xs, const float* __restrict__ rinit, const uint32_t* __restrict__ mask,
             const float* __restrict__ Qs, int G_arg, int64_t N, int B, int64_t n_steps, int steps_per_wg, int n_qb,
             float* __restrict__ gl_s, uint32_t* __restrict__ gl_i, uint32_t* __restrict__ gl_cnt, int64_t gl_cap,
             uint32_t* __restrict__ gthr, const int* __restrict__ gate) {
    // a gated launch (the device-memory re-pass, vdb_api.cpp): nothing to do when its count is 0
    if (gate && *gate == 0) return;
    constexpr int RT = RT_, NW = S2_NW;
    constexpr int QB = 32 * QT;
    constexpr int XPL = Planes<PREC>::XPL, QPL = 2;
    const int G = GC > 0 ? GC : G_arg;
    // query groups in flight (global query operand): PX, or VDB_S2_PQ when it divides PX (the
    // query block is L2-resident, so it needs less lead than the corpus stream)
#ifndef VDB_S2_PQ
#define VDB_S2_PQ 0
#endif
    constexpr int PQ = QLDS ? 1 : (VDB_S2_PQ > 0 && VDB_S2_PQ < PX && PX % (VDB_S2_PQ > 0 ? VDB_S2_PQ : 1) == 0 ? VDB_S2_PQ : PX);
    constexpr size_t GSTEP = 8 * BLOCK_FLOATS;  // query: consecutive groups of one super tile
    constexpr size_t PLANE = 4 * BLOCK_FLOATS;  // query: lo plane after hi
    constexpr size_t XGSTEP = corpus_gstep();   // corpus (vdb_common.h corpus_block)
    const size_t XPLANE = corpus_plane(G);
    static_assert(PX <= QG_EXTRA, "query prefetch deeper than the duplicated groups");
    __shared__ float s_sc[QB * CAP];
    __shared__ uint32_t s_ix[QB * CAP];
    __shared__ int s_cnt[QB];
    __shared__ float s_thr[QB];
    __shared__ int s_need, s_done;
    __shared__ uint32_t s_pend[NW][RT * QT][64];  // per wave and tile: each lane's entries left for a compaction round
    extern __shared__ __attribute__((aligned(16))) float s_q[];  // QLDS: [G][plane][QT][256]

    const int lane = threadIdx.x & 63;
    const int lane4 = lane * 4;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#ifdef VDB_STAMP
    const unsigned long long st_t0 = S2_NOW();
    unsigned long long st_pro = 0, st_k = 0, st_e = 0, st_fl = 0, st_a = 0, st_n = 0;
#endif
    int wg, qb;
    xcd_map(n_qb, wg, qb);
    if (threadIdx.x == 0) {
        s_need = 0;
        s_done = 0;
    }
    for (int i = threadIdx.x; i < QB; i += 64 * NW) {
        s_cnt[i] = 0;
        s_thr[i] = -INFINITY;
    }
    const float* Qbase = Qs + s2_blk((uint64_t)(qb * QT), 0, G + QG_EXTRA);
    if constexpr (QLDS) {
        for (int e = threadIdx.x; e < G * 2 * QT * 64; e += 64 * NW) {
            const int l = e & 63, qt = (e >> 6) % QT, pl = (e / (64 * QT)) & 1, g = e / (128 * QT);
            *(f32x4*)(s_q + (size_t)e * 4) = *(const f32x4*)(Qbase + g * GSTEP + pl * PLANE + qt * BLOCK_FLOATS + 4 * l);
        }
    }
    __syncthreads();

    constexpr int QPW = QB / NW;

    const int64_t s_begin = (int64_t)wg * steps_per_wg;
    const int64_t s_end = s_begin + steps_per_wg < n_steps ? s_begin + steps_per_wg : n_steps;

    f32x4 xr[PX][RT][XPL];
    f32x4 qr[PQ][QT][QPL];
    auto q_lds = [&](int g, f32x4 (&q)[QT][QPL]) {
#pragma unroll
        for (int qt = 0; qt < QT; ++qt)
#pragma unroll
            for (int pl = 0; pl < QPL; ++pl) q[qt][pl] = *(const f32x4*)(s_q + ((size_t)(g * 2 + pl) * QT + qt) * 256 + lane4);
    };
    if (s_begin < s_end) {
        const float* xs = Xs + corpus_block((uint64_t)((s_begin * NW + wv) * RT), 0, 0, G);
#pragma unroll
        for (int p = 0; p < PX; ++p)
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int pl = 0; pl < XPL; ++pl)
                    xr[p][rt][pl] = corpus_ld<NT>(xs + p * XGSTEP + pl * XPLANE + rt * BLOCK_FLOATS + lane4);
        if constexpr (!QLDS) {
#pragma unroll
            for (int p = 0; p < PQ; ++p)
#pragma unroll
                for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                    for (int pl = 0; pl < QPL; ++pl)
                        qr[p][qt][pl] = *(const f32x4*)(Qbase + p * GSTEP + pl * PLANE + qt * BLOCK_FLOATS + lane4);
        } else {
            q_lds(0, qr[0]);
        }
    }
    // the next step's shared bounds and (L2) accumulator start values, loaded one step ahead:
    // lanes 0-31 hold rinit of row 32 t + lane of each tile (the A column of the init MFMA)
    constexpr int NRI = METRIC == 1 ? RT : 1;
    auto load_epi = [&](int64_t st_, uint32_t (&g_)[QT], float (&r_)[NRI]) {
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
            const int qg = qb * QB + qt * 32 + (lane & 31);
            g_[qt] = qg < B ? gthr[qg] : 0u;
        }
        if constexpr (METRIC == 1) {
            const int64_t tt = (st_ * NW + wv) * RT;
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) r_[rt] = lane < 32 ? rinit[(tt + rt) * 32 + lane] : 0.0f;
        }
    };
    uint32_t gkn[QT];
    float rin[NRI];
    if (s_begin < s_end) load_epi(s_begin, gkn, rin);
    const float ones = lane < 32 ? 1.0f : 0.0f;  // B of the init MFMA: row k = 0 all ones

#ifdef VDB_STAMP
    st_pro = S2_NOW() - st_t0;
#endif
    for (int64_t s = s_begin; s < s_end; ++s) {
#ifdef VDB_STAMP
        st_a = S2_NOW();
        ++st_n;
#endif
        const int64_t t0 = (s * NW + wv) * RT;
        const float* xs = Xs + corpus_block((uint64_t)t0, 0, 0, G);
        const float* xn = (s + 1 < s_end) ? Xs + corpus_block((uint64_t)(t0 + NW * RT), 0, 0, G) : xs;
        f32x16 acc[RT][QT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int qt = 0; qt < QT; ++qt) {
#pragma unroll
                for (int v = 0; v < 16; ++v) acc[rt][qt][v] = 0.0f;
                if constexpr (METRIC == 1)  // acc[i][j] = rinit[row i] * 1 (exact)
                    acc[rt][qt] = __builtin_amdgcn_mfma_f32_32x32x2f32(rin[METRIC == 1 ? rt : 0], ones, acc[rt][qt], 0,
                                                                       0, 0);
            }
        uint32_t gk[QT];
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) gk[qt] = gkn[qt];

        // one group: MFMAs of slot p, then refill slot p with the group PX ahead (this step's,
        // or the next step's first groups); refills pinned right behind the MFMAs
        auto group = [&](const int p, const int g, const float* xsrc, const float* qsrc) {
if constexpr (QLDS) {
                f32x4 qn[1][QT][QPL];
                q_lds(g + 1 < G ? g + 1 : 0, qn[0]);
                group_mfma<PREC, RT, QT>(xr[p], qr[0], acc);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                    for (int pl = 0; pl < XPL; ++pl)
                        xr[p][rt][pl] = corpus_ld<NT>(xsrc + pl * XPLANE + rt * BLOCK_FLOATS + lane4);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                    for (int pl = 0; pl < QPL; ++pl) qr[0][qt][pl] = qn[0][qt][pl];
            } else {
                group_mfma<PREC, RT, QT>(xr[p], qr[p % PQ], acc);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                    for (int pl = 0; pl < XPL; ++pl)
                        xr[p][rt][pl] = corpus_ld<NT>(xsrc + pl * XPLANE + rt * BLOCK_FLOATS + lane4);
#pragma unroll
                for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                    for (int pl = 0; pl < QPL; ++pl)
                        qr[p % PQ][qt][pl] = *(const f32x4*)(qsrc + pl * PLANE + qt * BLOCK_FLOATS + lane4);
                __builtin_amdgcn_sched_barrier(0);
            }
        };
#if VDB_S2_ONELOOP
        // one loop, the tail's refill source selected inside (as scan8: a peeled tail gave the
        // accumulators a rotated register assignment and a shuffle through VGPRs every step)
        for (int gb = 0; gb < G; gb += PX) {
            const bool last = gb + PX >= G;
            if (last && s + 1 < s_end) load_epi(s + 1, gkn, rin);
#pragma unroll
            for (int p = 0; p < PX; ++p)
                group(p, gb + p, last ? xn + (size_t)p * XGSTEP : xs + (size_t)(gb + p + PX) * XGSTEP,
                      Qbase + (size_t)(gb + p + PQ) * GSTEP);
        }
#else
        int gb = 0;
        for (; gb < G - PX; gb += PX) {
#pragma unroll
            for (int p = 0; p < PX; ++p)
                group(p, gb + p, xs + (size_t)(gb + p + PX) * XGSTEP, Qbase + (size_t)(gb + p + PQ) * GSTEP);
        }
        if (s + 1 < s_end) load_epi(s + 1, gkn, rin);
#pragma unroll
        for (int p = 0; p < PX; ++p)
            group(p, gb + p, xn + (size_t)p * XGSTEP, Qbase + (size_t)(gb + p + PQ) * GSTEP);
#endif

#ifdef VDB_SCAN2_KLOOP_ONLY
        {  // diagnostic build (make variant): the K-loop alone, results are garbage
            float f = 0.0f;
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int qt = 0; qt < QT; ++qt) f += tile_max16(acc[rt][qt]);
            if (f == 1234.5f) gl_s[0] = f;
            continue;
        }
#endif
        // ---- epilogue: the accumulators are the scores (cosine) or half of them (L2) ----
#ifdef VDB_STAMP
        {
            const unsigned long long t = S2_NOW();
            st_k += t - st_a;
            st_a = t;
        }
#endif
        float thrh[QT];
        bool qok[QT];
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
            const int ql = qt * 32 + (lane & 31);
            const float thr = fmaxf(s_thr[ql], key_to_float(gk[qt]));
            thrh[qt] = METRIC == 0 ? thr : 0.5f * thr;
            qok[qt] = qb * QB + ql < B;
        }
        // The hot path: every tile's maximum against its threshold (wave-uniform bit rt QT + qt)
        uint32_t todo = 0;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
                todo |= __any(qok[qt] && tile_max16(acc[rt][qt]) > thrh[qt]) ? 1u << (rt * QT + qt) : 0u;
        // Insertion (as vdb_scan8_kernel.h): one passing tile at a time through ONE copy of the
        // code (its registers picked by a wave-uniform switch); each lane's pass bits from 16
        // independent compares, then one round per hit of the lane with the most hits -- with
        // one wave per SIMD a compare-ballot-branch chain per register cost ~140 cycles, ~2.9 K per
        // tile.  Only the lanes whose score passes append (one returning LDS atomic each);
        // entries that find the buffer full wait in s_pend for a compaction round.
        uint32_t pmask = 0;  // wave-uniform: tiles with entries left in s_pend
        for (bool joined = false;; joined = true) {
            while (todo != 0u) {
                const int t = __builtin_amdgcn_readfirstlane(__builtin_ctz(todo));
                todo &= todo - 1u;
                f32x16 h;
                switch (t) {
#define S2_TILE_CASE(T_)                                               \
    case T_:                                                           \
        if constexpr ((T_) < RT * QT) h = acc[(T_) / QT][(T_) % QT];   \
        break;
                    S2_TILE_CASE(0) S2_TILE_CASE(1) S2_TILE_CASE(2) S2_TILE_CASE(3)
                    S2_TILE_CASE(4) S2_TILE_CASE(5) S2_TILE_CASE(6) S2_TILE_CASE(7)
#undef S2_TILE_CASE
                    default: __builtin_unreachable();
                }
                static_assert(RT * QT <= 8, "tile switch covers 8 tiles");
                const int rt = t / QT, qt = t - rt * QT;
                const int ql = qt * 32 + (lane & 31);
                uint32_t gkq = gk[0];
                bool ok = qok[0];
#pragma unroll
                for (int q2 = 1; q2 < QT; ++q2)
                    if (qt == q2) {
                        gkq = gk[q2];
                        ok = qok[q2];
                    }
                const float thr = fmaxf(s_thr[ql], key_to_float(gkq));
                const float th = METRIC == 0 ? thr : 0.5f * thr;
                const uint32_t cand = joined ? s_pend[wv][t][lane] : ok ? tile_valid16(mask, t0 + rt, N, lane) : 0u;
                const uint32_t rb = (uint32_t)((t0 + rt) * 32) + 4u * (uint32_t)(lane >> 5);
                uint32_t pm = 0;
#pragma unroll
                for (int v = 0; v < 16; ++v) pm |= (h[v] > th ? 1u : 0u) << v;
                pm &= cand;
                uint32_t left = 0;
                while (__any(pm != 0u)) {
                    if (pm != 0u) {
                        const int v = __builtin_ctz(pm);
                        pm &= pm - 1u;
                        float a_ = h[0];
#pragma unroll
                        for (int u = 1; u < 16; ++u) a_ = v == u ? h[u] : a_;
                        const float sc = METRIC == 0 ? a_ : 2.0f * a_;
                        const int pos = atomicAdd(&s_cnt[ql], 1);
                        if (pos < CAP) {
                            s_sc[ql * CAP + pos] = sc;
                            s_ix[ql * CAP + pos] = rb + (uint32_t)((v & 3) + 8 * (v >> 2));
                        } else {
                            left |= 1u << v;
                        }
                    }
                }
                if (__any(left != 0u)) {
                    s_pend[wv][t][lane] = left;
                    pmask |= 1u << t;
                }
            }
            // compaction rounds (vdb_scan.hip): lockstep = one workgroup barrier per step;
            // FLAGSYNC = a wave with leftovers raises s_need and the others join at their step end
            if constexpr (!FLAGSYNC) {
                if (!__syncthreads_or(pmask != 0u)) break;
            } else {
                const bool mine = pmask != 0u;
                if (mine && lane == 0) lds_flag_st(&s_need, 1);
                if (!mine && (joined || !__builtin_amdgcn_readfirstlane(lds_flag_ld(&s_need)))) break;
                __syncthreads();  // B1
            }
            for (int q = wv; q < QB; q += NW)
                if (s_cnt[q] >= CAP)
                    compact_query<KW, CAP>(s_sc + q * CAP, s_ix + q * CAP, s_cnt + q, s_thr + q,
                                           KW == KP && qb * QB + q < B ? gthr + qb * QB + q : nullptr);
            if (FLAGSYNC && threadIdx.x == 0) lds_flag_st(&s_need, 0);
            __syncthreads();  // B2
            todo = pmask;
            pmask = 0;
        }
#ifdef VDB_STAMP
        {
            const unsigned long long t = S2_NOW();
            st_e += t - st_a;
            st_a = t;
        }
#endif
    }
#ifdef VDB_STAMP
    st_a = S2_NOW();
#endif

    // FLAGSYNC: keep answering compaction rounds until every wave is past its last step
    if (FLAGSYNC && lane == 0) atomicAdd(&s_done, 1);
    for (; FLAGSYNC;) {
        if (lane == 0) lds_flag_st(&s_need, 1);
        __syncthreads();  // B1
        if (__builtin_amdgcn_readfirstlane(lds_flag_ld(&s_done)) == NW) break;
        for (int q = wv; q < QB; q += NW)
            if (s_cnt[q] >= CAP)
                compact_query<KW, CAP>(s_sc + q * CAP, s_ix + q * CAP, s_cnt + q, s_thr + q,
                                       KW == KP && qb * QB + q < B ? gthr + qb * QB + q : nullptr);
        if (threadIdx.x == 0) lds_flag_st(&s_need, 0);
        __syncthreads();  // B2
    }

    // ---- flush: entries above the shared bound -> global per-query lists ----
    __syncthreads();
    uint32_t tkey = 0;
    if (lane < QPW && qb * QB + wv + NW * lane < B) {
        const int q = wv + NW * lane;
        uint32_t dk = 0;
        if (KW < KP && s_begin < s_end) {  // this workgroup's drop bound (its KW-th best, once compacted)
            dk = s_thr[q] == -INFINITY ? 0u : order_key(s_thr[q]);
            if (dk) atomicMax(gthr + qb * QB + q, dk);
        }
        tkey = max(gthr[qb * QB + q], dk);
    }
    append_flush<CAP>(s_sc, s_ix, s_cnt, wv, NW, QPW, qb * QB, B, tkey, gl_s, gl_i, gl_cnt, gl_cap);
#ifdef VDB_STAMP
    {
        const unsigned long long t = S2_NOW();
        st_fl = t - st_a;
        const int w = blockIdx.x * NW + wv;
        if (lane == 0 && w < (1 << 16)) {
            g_scan2_stamps[w][0] = st_pro;
            g_scan2_stamps[w][1] = st_k;
            g_scan2_stamps[w][2] = st_e;
            g_scan2_stamps[w][3] = t - st_t0;
            g_scan2_stamps[w][4] = 0;
            g_scan2_stamps[w][5] = st_fl;
            g_scan2_stamps[w][6] = st_n;
            g_scan2_stamps[w][7] = st_t0;
        }
    }
#endif
}


// ---- launch templates ----
inline int scan2_qb(int KP) { return KP == 256 ? 32 : 64; }

// The query block goes to LDS when it is small (C4: 64 queries x 128 dims = 32 KiB; the
// 128-query shape: 64 KiB).
inline bool scan2_qlds(int G16, int KP, bool q4 = false) {
    return (size_t)G16 * 2 * (q4 ? 4 : scan2_qb(KP) / 32) * 1024 <= (q4 ? 64 : 32) * 1024;
}

template <int P, int M, int QT, int PX, int KP, int CAP, bool NT, bool QL, bool FS, int GC, int RT_ = S2_RT,
          int KW = KP>
static hipError_t scan2_launch_g(const float* Xs, const float* rinit, const uint32_t* mask, const float* Qs, int G,
                                 int64_t N, int B, int n_qblocks, int64_t n_steps, int n_wg, int spw, float* gl_s,
                                 uint32_t* gl_i, uint32_t* gl_cnt, int64_t gl_cap, uint32_t* gthr, const int* gate,
                                 hipStream_t st) {
    auto k = scan2_kernel<P, M, QT, PX, KP, CAP, NT, QL, FS, GC, RT_, KW>;
    const size_t lds = QL ? (size_t)G * 2 * QT * 1024 : 0;
    if (QL) {
        // the dynamic part (query block) plus the static top-k buffers must fit the 160 KiB of a
        // CU: raise the dynamic limit to what this call needs (monotone; racing calls only
        // raise it to values that fit)
        static std::atomic<size_t> lds_set{0};
        size_t cur = lds_set.load();
        while (lds > cur) {
            hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
            if (lds_set.compare_exchange_weak(cur, lds)) break;
        }
    }
    const int n_wg8 = (n_wg + 7) / 8 * 8;
    hipLaunchKernelGGL(k, dim3(n_wg8 * n_qblocks), dim3(64 * S2_NW), lds, st, Xs, rinit, mask, Qs, G, N, B, n_steps, spw,
                       n_qblocks, gl_s, gl_i, gl_cnt, gl_cap, gthr, gate);
    return hipGetLastError();
}

// query block in LDS (short rows): the common short row (D = 128 -> 8 groups) gets its own
// instantiation with the group count built in
template <int P, int M, int QT, int PX, int KP, int CAP, bool NT, bool QL, bool FS, int RT_ = S2_RT, int KW = KP>
static hipError_t scan2_launch(const float* Xs, const float* rinit, const uint32_t* mask, const float* Qs, int G,
                               int64_t N, int B, int n_qblocks, int64_t n_steps, int n_wg, int spw, float* gl_s,
                               uint32_t* gl_i, uint32_t* gl_cnt, int64_t gl_cap, uint32_t* gthr, const int* gate,
                               hipStream_t st) {
    if constexpr (QL) {
        if (G == 8)
            return scan2_launch_g<P, M, QT, PX, KP, CAP, NT, QL, FS, 8, RT_, KW>(
                Xs, rinit, mask, Qs, G, N, B, n_qblocks, n_steps, n_wg, spw, gl_s, gl_i, gl_cnt, gl_cap, gthr, gate, st);
    }
    return scan2_launch_g<P, M, QT, PX, KP, CAP, NT, QL, FS, 0, RT_, KW>(
        Xs, rinit, mask, Qs, G, N, B, n_qblocks, n_steps, n_wg, spw, gl_s, gl_i, gl_cnt, gl_cap, gthr, gate, st);
}

// The argument list of one (precision, metric) unit's launcher (launch_scan2 dispatches).
#define S2_UNIT_PARAMS                                                                                             \
    int KP, const float *Xs, const float *rinit, const uint32_t *mask, const float *Qs, int G, int64_t N, int B,    \
        int n_qblocks, int64_t n_steps, int n_wg, int spw, float *gl_s, uint32_t *gl_i, uint32_t *gl_cnt,          \
        int64_t gl_cap, uint32_t *gthr, bool nt, bool ql, bool fs, bool q4, const int *gate, hipStream_t st
#define S2_ARGS Xs, rinit, mask, Qs, G, N, B, n_qblocks, n_steps, n_wg, spw, gl_s, gl_i, gl_cnt, gl_cap, gthr, gate, st
#define S2_ONE(P, M, KPV, QTV, PXV, CAPV, NTV, QLV, FSV)                 \
    if (KP == KPV && nt == NTV && ql == QLV && fs == FSV && !q4) \
        return scan2_launch<P, M, QTV, PXV, KPV, CAPV, NTV, QLV, FSV>(S2_ARGS);
// the 128-query shape (query block in LDS, 2 row tiles per wave, KW = 48 kept of KP = 128)
#define S2_ONE4(P, M, PXV, FSV)                                               \
    if (KP == 128 && ql && fs == FSV && q4)                                   \
        return scan2_launch<P, M, 4, PXV, 128, 64, false, true, FSV, 2, 48>(S2_ARGS);
#define S2_KP(P, M, PXV, NTV, QLV, FSV)                    \
    S2_ONE(P, M, 32, 2, PXV, 128, NTV, QLV, FSV)           \
    S2_ONE(P, M, 64, 2, PXV, 128, NTV, QLV, FSV)           \
    S2_ONE(P, M, 128, 2, PXV, 192, NTV, QLV, FSV)          \
    S2_ONE(P, M, 256, 1, PXV, 320, NTV, QLV, FSV)
// PX (corpus groups in flight): bf16x3 2 (query operand in registers too), 4 with the query
// block in LDS; bf16 (half the corpus registers per group) 4
#define S2_MODES(P, M, PXV, PXL)                                                   \
    S2_KP(P, M, PXV, false, false, false) S2_KP(P, M, PXV, true, false, false)     \
    S2_KP(P, M, PXL, false, true, false) S2_KP(P, M, PXL, false, true, true)       \
    S2_KP(P, M, PXV, false, false, true) S2_KP(P, M, PXV, true, false, true)       \
    S2_ONE4(P, M, PXL, false) S2_ONE4(P, M, PXL, true)
#ifndef VDB_S2_QLDS_PX
#define VDB_S2_QLDS_PX 2
#endif
// One instantiation unit: every (KP, nt, qlds, step end) variant of precision P, metric M.
#define S2_UNIT(NAME, P, M, PXV, PXL)                 \
    hipError_t NAME(S2_UNIT_PARAMS) {                 \
        S2_MODES(P, M, PXV, PXL)                      \
        return hipErrorInvalidValue;                  \
    }
hipError_t launch_scan2_b3c(S2_UNIT_PARAMS);
hipError_t launch_scan2_b3l(S2_UNIT_PARAMS);
hipError_t launch_scan2_b1c(S2_UNIT_PARAMS);
hipError_t launch_scan2_b1l(S2_UNIT_PARAMS);

}  // namespace vdb

#ifdef VDB_STAMP
#define S2_STAMP_READER(SFX)                                                                                \
    extern "C" int vdb_debug_scan2_stamps_##SFX(unsigned long long* out, int n_waves) {                     \
        return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(vdb::g_scan2_stamps),                                \
                                        (size_t)n_waves * 8 * sizeof(unsigned long long));                  \
    }
#else
#define S2_STAMP_READER(SFX)
#endif
