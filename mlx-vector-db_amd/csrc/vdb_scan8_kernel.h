// vdb_scan8_kernel.h — the int8 candidate pass (PREC_I8 / PREC_I8Q / PREC_I8X3) and its launch templates
// (included by vdb_scan8.hip and the per-(precision, metric) instantiation units
// vdb_scan8_{i1,i3}{c,l}.hip, which the build compiles in parallel).
//
// Arithmetic.  The candidate copy holds the CENTRED rows z = y - mu (y the row the pass scores:
// cosine the normalised row, L2 the row; mu the mean row of the first add, vdb_api.cpp) as
// 16-bit fixed point in two int8 planes, z ~ s_x (xh + xl / 256) (vdb_scan8.hip quant_rows).
// The query block q (cosine: normalised) is quantised the same way per batch, q ~ s_q (qh + ql /
// 256) (vdb_scan8.hip prep8).  Per 32-dim group and (row tile, query tile) the pass issues
//   PREC_I8    xh.qh -> H                                   1 v_mfma_i32_32x32x32_i8
//   PREC_I8Q   xh.qh -> H, xh.ql -> L                       2 (the 8-bit corpus x the 16-bit query)
//   PREC_I8X3  xh.qh -> H, xh.ql + xl.qh -> L               3 v_mfma_i32_32x32x32_i8
// and the (half-)score is H s_x s_q (+ L s_x s_q / 256): integer sums are exact, an i8 MFMA does
// twice the K of a bf16 one in the same cycles, and the I8 pass reads one byte per element
// (half of the bf16 hi plane) and one accumulator set (scan2's register shape: 4 row tiles per
// wave).  Its error bound is the wider one (the query's 8-bit rounding |z~.(q - s_q qh)| adds
// to the corpus term), which the finish's exact-key certificate (vdb_exact.hip: the exact k-th
// best candidate against acut + eps, one eps instead of two) absorbs at C2 / C6's gaps; where
// it does not, auto re-passes the query in I8X3.  Ranking by z.q instead of y.q drops mu.q, the same for every
// row of a query, so candidates, bounds and the certificate (all differences of approximate
// scores) are unchanged by it.  L2 scores q.x - |x|^2/2 = q.mu + q.z - |x|^2/2: H starts at
// rint(-|x|^2 / 2 / (s_x s_q)) per row, so the pass ends at score / 2 (up to q.mu).
// Error vs the exact score (finish_kernel's eps, vdb_api.cpp): the corpus rounding
// |q.(z - z~)| (the measured row residuals, Cauchy-Schwarz or along the residual direction, as
// for bf16), the query rounding |z~.(q - q~)| and for I8X3 the dropped xl.ql term (per query,
// prep8 -> qerr), the L2 start rounding, and fp32 rounding of the final combination.
//
// Shape: scan2's (4 waves, one per SIMD, a shared query block of QT tiles, RT row tiles per
// wave and step -- I8 4, I8X3 2: two accumulator sets per tile --, PX corpus groups in flight in
// registers, the query block from L2 or, for short rows, LDS).  Epilogue: a tile passes when its
// largest H clears the query's threshold in H units (I8X3: minus the largest |L| term, lsl per
// query), then the fp32 score of each register is compared and appended.
#pragma once
#include "vdb_scan2_kernel.h"

namespace vdb {

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

// waves per workgroup (one workgroup per CU: 4 = one wave per SIMD with all its registers;
// 8 = two, 256 registers each, one wave's epilogue under the other's K-loop -- A/B build define)
#ifndef VDB_S8_NW
#define VDB_S8_NW 4
#endif
constexpr int S8_NW = VDB_S8_NW;
// the I8X3 L2 pass's own wave count: 8 waves, two per SIMD, one wave's epilogue under the other's
// K-loop (C4 scan 2.92 -> 2.77 ms, +4% QPS, profiles/r04_ab/x8; build define, 4 = the old shape).
// The others keep S8_NW = 4 (8 waves there: C2 -15%, C3 -25%, C6 -6%, profiles/r04_ab/nw8).
#ifndef VDB_S8_NW_X3L
#define VDB_S8_NW_X3L 8
#endif
constexpr int scan8_nw(int prec, int metric, int QT = 2) {
    return (prec == PREC_I8X3 || prec == PREC_I8Q) && metric == 1 && QT != 4 ? VDB_S8_NW_X3L : S8_NW;
}
// the step's group loop: one loop with the tail selected inside (1) or the tail peeled (0)
// the corpus loads non-temporal with the query block in LDS (one query block, flag-gated): C6
// scan 0.243 -> 0.219 ms, C2 (with the block in LDS past 16 groups) 0.148 -> 0.143 ms
// (profiles/r05_ab/ab8_ntql.log; before, only the L2-operand shapes loaded nt)
#ifndef VDB_S8_NTQL
#define VDB_S8_NTQL 1
#endif
#ifndef VDB_S8_ONELOOP
#define VDB_S8_ONELOOP 0
#endif
// the epilogue's insertions: the step's thresholds reused in the first round and one round per
// wave-uniform register index (1), or thresholds re-read and a per-lane select per hit (0)
#ifndef VDB_S8_INS2
#define VDB_S8_INS2 0
#endif
// the first round's thresholds alone (the per-lane select kept)
#ifndef VDB_S8_INSTHR
#define VDB_S8_INSTHR 0
#endif

#ifdef VDB_STAMP8
// Diagnostic build only (make variant VDEFS=-DVDB_STAMP8): per-wave cycles of scan8_kernel:
// [0] total, [1] in the stream waits (s8_wait), [2] K-loop (step start to the last group's
// refill, waits included), [3] epilogue, [4] steps, [5] start time (absolute)
static __device__ unsigned long long g_scan8_stamps[1 << 16][12];
#define S8_NOW() __builtin_amdgcn_s_memtime()
#define S8_STAMP(...) __VA_ARGS__
#else
#define S8_STAMP(...)
#endif
// row tiles per wave per step: I8 cosine 4 (one accumulator set, 128 registers), I8X3 2 (two
// sets), I8 L2 2 (its per-row start values, prefetched a step ahead, would spill at 4)
#ifndef VDB_S8_RT1
#define VDB_S8_RT1 4
#endif
#ifndef VDB_S8_RT3
#define VDB_S8_RT3 2
#endif
// (the 8-wave I8X3 L2 shape: one row tile per wave, the same rows per step with 256 registers)
constexpr int scan8_rt(int prec, int metric) {
    return (prec == PREC_I8X3 || prec == PREC_I8Q) && metric == 1 && VDB_S8_NW_X3L == 8 ? 1
           : prec == PREC_I8X3 || prec == PREC_I8Q || metric == 1                   ? VDB_S8_RT3
                                                                : VDB_S8_RT1;
}
constexpr int scan8_rows(int prec, int metric) { return scan8_rt(prec, metric) * scan8_nw(prec, metric) * 32; }

template <int PREC>
struct Planes8 {
    static constexpr int XPL = PREC == PREC_I8X3 ? 2 : 1;                       // corpus planes read
    static constexpr int QPL = PREC == PREC_I8X3 || PREC == PREC_I8Q ? 2 : 1;   // query planes read
    static constexpr bool L = PREC == PREC_I8X3 || PREC == PREC_I8Q;            // the L accumulator set
};

template <int PREC, int RT, int QT>
__device__ __forceinline__ void group_mfma8(const f32x4 (&x)[RT][Planes8<PREC>::XPL],
                                            const f32x4 (&q)[QT][Planes8<PREC>::QPL], i32x16 (&aH)[RT][QT],
                                            i32x16 (&aL)[RT][QT]) {
    // every H product first, then the L ones (I8X3): the tile tests after the step's last group
    // read H alone, so H is complete while the group's L MFMAs still run; and each L set's two
    // dependent MFMAs are not issued back to back
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int qt = 0; qt < QT; ++qt)
            aH[rt][qt] = __builtin_amdgcn_mfma_i32_32x32x32_i8(__builtin_bit_cast(i32x4, x[rt][0]),
                                                               __builtin_bit_cast(i32x4, q[qt][0]), aH[rt][qt], 0, 0, 0);
    if constexpr (PREC == PREC_I8Q) {  // L = xh.ql alone (the corpus's 8 bits)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
                aL[rt][qt] = __builtin_amdgcn_mfma_i32_32x32x32_i8(
                    __builtin_bit_cast(i32x4, x[rt][0]), __builtin_bit_cast(i32x4, q[qt][Planes8<PREC>::QPL - 1]),
                    aL[rt][qt], 0, 0, 0);
    }
    if constexpr (PREC == PREC_I8X3) {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
                aL[rt][qt] = __builtin_amdgcn_mfma_i32_32x32x32_i8(
                    __builtin_bit_cast(i32x4, x[rt][0]), __builtin_bit_cast(i32x4, q[qt][Planes8<PREC>::QPL - 1]),
                    aL[rt][qt], 0, 0, 0);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
                aL[rt][qt] = __builtin_amdgcn_mfma_i32_32x32x32_i8(
                    __builtin_bit_cast(i32x4, x[rt][Planes8<PREC>::XPL - 1]), __builtin_bit_cast(i32x4, q[qt][0]),
                    aL[rt][qt], 0, 0, 0);
    }
}

// the sum of 16 accumulators mod 2^32 as a depth-3 tree of v_add3_u32 (the checksum)
__device__ __forceinline__ uint32_t hsum16(const i32x16& a) {
    const uint32_t s0 = (uint32_t)a[0] + (uint32_t)a[1] + (uint32_t)a[2];
    const uint32_t s1 = (uint32_t)a[3] + (uint32_t)a[4] + (uint32_t)a[5];
    const uint32_t s2 = (uint32_t)a[6] + (uint32_t)a[7] + (uint32_t)a[8];
    const uint32_t s3 = (uint32_t)a[9] + (uint32_t)a[10] + (uint32_t)a[11];
    const uint32_t s4 = (uint32_t)a[12] + (uint32_t)a[13] + (uint32_t)a[14];
    return (s0 + s1 + s2) + (s3 + s4 + (uint32_t)a[15]);
}

__device__ __forceinline__ int imax16(const i32x16& a) {  // a depth-3 tree of v_max3_i32
    const int m0 = max(max(a[0], a[1]), a[2]), m1 = max(max(a[3], a[4]), a[5]), m2 = max(max(a[6], a[7]), a[8]);
    const int m3 = max(max(a[9], a[10]), a[11]), m4 = max(max(a[12], a[13]), a[14]);
    return max(max(max(m0, m1), m2), max(max(m3, m4), a[15]));
}

// The streams the K-loop consumes -- corpus tiles, global query tiles, L2 start values -- are
// loaded by inline asm the compiler does not track, and waited for explicitly: s_waitcnt
// vmcnt(N), N = this kernel's loads issued after the slot (a compile-time constant), tied to
// the registers the slot fills.  Compiler-visible loads carried across the step loop made its
// wait pass drain every outstanding load at the loop header (s_waitcnt vmcnt(0) before the
// first MFMA of each step, the whole next-step prefetch included).  vmcnt retires in issue
// order, so any other younger memory operation only makes a wait more conservative.
template <bool NT>
__device__ __forceinline__ f32x4 s8_ld(const float* base, uint32_t voff) {
    f32x4 r;
    if constexpr (NT)
        asm volatile("global_load_dwordx4 %0, %1, %2 nt" : "=v"(r) : "v"(voff), "s"(base));
    else
        asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(r) : "v"(voff), "s"(base));
    return r;
}
template <int N, int A, int C>
__device__ __forceinline__ void s8_wait(f32x4 (&r)[A][C]) {
    asm volatile("s_waitcnt vmcnt(%1)" : "+v"(r[0][0]) : "n"(N));
#pragma unroll
    for (int a = 0; a < A; ++a)
#pragma unroll
        for (int c = 0; c < C; ++c)
            if (a + c > 0) asm volatile("" : "+v"(r[a][c]));
}
template <int A, int C>
__device__ __forceinline__ void s8_tie(f32x4 (&r)[A][C]) {  // after an s8_wait: these are ready too
#pragma unroll
    for (int a = 0; a < A; ++a)
#pragma unroll
        for (int c = 0; c < C; ++c) asm volatile("" : "+v"(r[a][c]));
}


// The smallest H that can still pass threshold th (half units) given |L uL| <= slack, minus a
// margin for the fp32 evaluation: H <= the result means the tile's scores are all <= th.
__device__ __forceinline__ int h_floor(float th, float slack, float invU) {
    // (selects, not branches: the compiler made each test an exec-mask branch, three per query tile
    // and step)
    const float t = (th - slack) * invU;
    const float m = t - fabsf(t) * 1e-5f - 4.0f;
    const int r = (int)floorf(fminf(fmaxf(m, -2.0e9f), 2.0e9f));
    return th > -INFINITY && m > -2.0e9f ? r : INT_MIN;
}

// Per-batch scalars written by prep8 (device): [0] uH = s_x s_q, [1] uL = uH / 256, [2] 1 / uH.
template <int PREC, int METRIC, int QT, int PX, int KP, int CAP, bool NT, bool QLDS, bool FLAGSYNC, int GC = 0,
          int RT_ = scan8_rt(PREC, METRIC), int KW = KP>
__global__ void __launch_bounds__(64 * scan8_nw(PREC, METRIC, QT), 1)
scan8_kernel(const float* __restrict__ Xq, const float* __restrict__ rinit, const uint32_t* __restrict__ mask,
             const float* __restrict__ Qq, const float* __restrict__ lsl, const float* __restrict__ qscal, int G_arg,
             int64_t N, int B, int64_t n_steps, int steps_per_wg, int n_qb, float* __restrict__ gl_s,
             uint32_t* __restrict__ gl_i, uint32_t* __restrict__ gl_cnt, int64_t gl_cap, uint32_t* __restrict__ gthr,
             const int* __restrict__ gate, uint32_t* __restrict__ chkp, int chk_ld, int chk_l) {
    // a gated launch (the device-memory re-pass, vdb_api.cpp): nothing to do when its count is 0
    if (gate && *gate == 0) return;
    constexpr int RT = RT_, NW = scan8_nw(PREC, METRIC, QT);
    constexpr int QB = 32 * QT;
    constexpr int XPL = Planes8<PREC>::XPL, QPL = Planes8<PREC>::QPL;
    constexpr bool HL = Planes8<PREC>::L;
    const int G = GC > 0 ? GC : G_arg;
    constexpr int PQ = QLDS ? 1 : PX;
    constexpr int LQP = QPL;  // planes of the query block in LDS (I8 reads qh alone)
    constexpr size_t GSTEP = 8 * BLOCK_FLOATS;  // query: consecutive groups of one super tile
    constexpr size_t PLANE = 4 * BLOCK_FLOATS;  // query: lo plane after hi
    constexpr size_t XGSTEP = corpus_gstep();
    const size_t XPLANE = corpus_plane(G);
    static_assert(PX <= QG_EXTRA, "query prefetch deeper than the duplicated groups");
    __shared__ float s_sc[QB * CAP];
    __shared__ uint32_t s_ix[QB * CAP];
    __shared__ int s_cnt[QB];
    __shared__ float s_thr[QB];
    __shared__ int s_need, s_done;
    __shared__ uint32_t s_chk[HL ? 2 : 1][QB];  // the checksum's per-query sums of this workgroup
    __shared__ uint32_t s_pend[NW][8][64];  // per wave and tile: each lane's entries left for a compaction round
    extern __shared__ __attribute__((aligned(16))) float s_q[];  // QLDS: [G][LQP planes][QT][256]

    const int lane = threadIdx.x & 63;
    const int lane4 = lane * 4;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    S8_STAMP(const unsigned long long st_t0 = S8_NOW(), st_r0 = __builtin_amdgcn_s_memrealtime(); unsigned long long st_w = 0, st_k = 0, st_e = 0, st_n = 0, st_x = 0, st_y = 0, st_z = 0, st_q = 0, st_f = 0;)
    int wg, qb;
    xcd_map(n_qb, wg, qb);
    if (threadIdx.x == 0) {
        s_need = 0;
        s_done = 0;
    }
    for (int i = threadIdx.x; i < QB; i += 64 * NW) {
        s_cnt[i] = 0;
        s_thr[i] = -INFINITY;
        s_chk[0][i] = 0u;
        if constexpr (HL) s_chk[HL ? 1 : 0][i] = 0u;
    }
    const float uH = qscal[0], uL = qscal[1], invU = qscal[2];
    float qsl[QT];  // per query: bound of |L uL| (the prefilter's slack)
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
        const int qg = qb * QB + qt * 32 + (lane & 31);
        qsl[qt] = qg < B ? lsl[qg] : 0.0f;
    }
    const float* Qbase = Qq + s2_blk((uint64_t)(qb * QT), 0, G + QG_EXTRA);
    if constexpr (QLDS) {
        for (int e = threadIdx.x; e < G * LQP * QT * 64; e += 64 * NW) {
            const int l = e & 63, qt = (e >> 6) % QT, pl = (e / (64 * QT)) % LQP, g = e / (64 * QT * LQP);
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
            for (int pl = 0; pl < QPL; ++pl) q[qt][pl] = *(const f32x4*)(s_q + ((size_t)(g * LQP + pl) * QT + qt) * 256 + lane4);
    };
    // The shared bound is read once: with KW < KP (the I8 shape) nothing raises it during the
    // scan but the pilot (before it); with KW == KP other workgroups' compactions do, and a
    // stale copy only drops fewer rows (same speed, measured: profiles/r03_i8/)
    uint32_t gk[QT];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) gk[qt] = gthr[qb * QB + qt * 32 + (lane & 31)];
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the compiler's loads are done before the streams start
    // loads per slot (group) of the streams: corpus tiles, + query tiles from global memory
    constexpr int LPS = RT * XPL + (QLDS ? 0 : QT * QPL);
    // loads issued after a step's start values (for the next step) within that step: the tail
    // groups' refills after the first (one loop: all of them)
    constexpr int RIN_YOUNGER = VDB_S8_ONELOOP ? PX * LPS : (PX - 1) * LPS;
    const uint32_t voff = (uint32_t)lane * 16u;
    // L2: the next step's start values (the batch's integer H starts, vdb_scan8.hip rstart8), loaded
    // one step ahead, before the tail groups' refills
    // (lane half h holds -|x|^2/2 of rows 32 t + 8 a + 4 h + b, a, b = 0..3, of each tile: the
    // rows of its accumulator registers 4 a + b)
    constexpr int NRI = METRIC == 1 ? RT : 1;
    auto load_epi = [&](int64_t st_, f32x4 (&r_)[NRI][4]) {
        if constexpr (METRIC == 1) {
            const int64_t tt = (st_ * NW + wv) * RT;
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int a = 0; a < 4; ++a)
                    r_[rt][a] = s8_ld<false>(rinit + (tt + rt) * 32 + 8 * a, (uint32_t)(lane >> 5) * 16u);
        }
    };
    f32x4 rin[NRI][4];
    // The checksum (ABFT, vdb_scan8.hip): per lane and query tile, the sum (mod 2^32) of every H
    // (and L) accumulator of rows < N this wave produced -- the same registers the tile tests read
    uint32_t ckh[QT], ckl[QT];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) ckh[qt] = ckl[qt] = 0u;
    if (s_begin < s_end) {
        load_epi(s_begin, rin);  // before the slots: PX * LPS loads younger than these
        const float* xs = Xq + corpus_block((uint64_t)((s_begin * NW + wv) * RT), 0, 0, G);
#pragma unroll
        for (int p = 0; p < PX; ++p) {
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int pl = 0; pl < XPL; ++pl)
                    xr[p][rt][pl] = s8_ld<NT>(xs + p * XGSTEP + pl * XPLANE + rt * BLOCK_FLOATS, voff);
            if constexpr (!QLDS) {
#pragma unroll
                for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                    for (int pl = 0; pl < QPL; ++pl)
                        qr[p][qt][pl] = s8_ld<false>(Qbase + p * GSTEP + pl * PLANE + qt * BLOCK_FLOATS, voff);
            }
        }
        if constexpr (QLDS) q_lds(0, qr[0]);
        // L2 start values: waited for here, inside the block that loads them, and again at the
        // end of every step (below) -- never carried in flight across a join or the loop header.
        // The compiler may copy a value at a join (phi copies: seen at the loop header of the I8 /
        // I8X3 L2 QLDS kernels and after this block in the 128-query shape, tools/vmcnt_check.py),
        // and a copy of a register an asm load is still filling reads stale data (a
        // cold first search returned wrong, certified L2 results).  Free in time: the first group
        // waits for the slots issued after these loads anyway.
        if constexpr (METRIC == 1) s8_wait<PX * LPS>(rin);
    }

    // The tile tests' integer thresholds (flag-gated shapes with the query block in LDS): computed
    // here and again after each compaction round this wave takes part in -- nothing else changes
    // s_thr (gk is read once) -- not in every step's epilogue (an LDS read and ~20 vector
    // instructions per query tile and step).  (The other shapes recompute them per step: carried
    // across the loop there, the extra live registers moved asm-loaded slots through AGPRs before
    // their waits, tools/vmcnt_check.py.)
    constexpr bool THC = FLAGSYNC && QLDS;
    int thc[QT];
    auto thr_of = [&](int qt, float& thf_) {
        const int ql = qt * 32 + (lane & 31);
        const float thr = fmaxf(s_thr[ql], key_to_float(gk[qt]));
        thf_ = METRIC == 0 ? thr : 0.5f * thr;
        return h_floor(thf_, qsl[qt], invU);
    };
    auto refresh_thr = [&]() {
        if constexpr (THC) {
#pragma unroll
            for (int qt = 0; qt < QT; ++qt) {
                float f;
                thc[qt] = thr_of(qt, f);
            }
        }
    };
    refresh_thr();
    for (int64_t s = s_begin; s < s_end; ++s) {
        S8_STAMP(const unsigned long long st_a = S8_NOW(); ++st_n;)
        const int64_t t0 = (s * NW + wv) * RT;
        const float* xs = Xq + corpus_block((uint64_t)t0, 0, 0, G);
        const float* xn = (s + 1 < s_end) ? Xq + corpus_block((uint64_t)(t0 + NW * RT), 0, 0, G) : xs;
        i32x16 aH[RT][QT], aL[RT][QT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            i32x16 init;
#pragma unroll
            for (int v = 0; v < 16; ++v) init[v] = 0;
            if constexpr (METRIC == 1) {
#pragma unroll
                for (int a = 0; a < 4; ++a)
#pragma unroll
                    for (int b2 = 0; b2 < 4; ++b2) init[4 * a + b2] = __float_as_int(rin[METRIC == 1 ? rt : 0][a][b2]);
            }
#pragma unroll
            for (int qt = 0; qt < QT; ++qt) {
                aH[rt][qt] = init;
#pragma unroll
                for (int v = 0; v < 16; ++v) aL[rt][qt][v] = 0;
            }
        }

        auto group = [&](const int p, const int g, const float* xsrc, const float* qsrc) {
            // slot p was filled PX - 1 slots (and, for a tail group, the L2 start values) ago
            S8_STAMP(const unsigned long long st_b = S8_NOW();)
            s8_wait<(PX - 1) * LPS>(xr[p]);
            S8_STAMP(st_w += S8_NOW() - st_b;)
            if constexpr (QLDS) {
                f32x4 qn[1][QT][QPL];
                q_lds(g + 1 < G ? g + 1 : 0, qn[0]);
                group_mfma8<PREC, RT, QT>(xr[p], qr[0], aH, aL);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                    for (int pl = 0; pl < XPL; ++pl)
                        xr[p][rt][pl] = s8_ld<NT>(xsrc + pl * XPLANE + rt * BLOCK_FLOATS, voff);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                    for (int pl = 0; pl < QPL; ++pl) qr[0][qt][pl] = qn[0][qt][pl];
                (void)qsrc;
            } else {
                s8_tie(qr[p % PQ]);  // loaded right after slot p's corpus tiles
                group_mfma8<PREC, RT, QT>(xr[p], qr[p % PQ], aH, aL);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                    for (int pl = 0; pl < XPL; ++pl)
                        xr[p][rt][pl] = s8_ld<NT>(xsrc + pl * XPLANE + rt * BLOCK_FLOATS, voff);
#pragma unroll
                for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                    for (int pl = 0; pl < QPL; ++pl)
                        qr[p % PQ][qt][pl] = s8_ld<false>(qsrc + pl * PLANE + qt * BLOCK_FLOATS, voff);
                __builtin_amdgcn_sched_barrier(0);
            }
        };
#if VDB_S8_ONELOOP
        // One loop over all groups, the last PX of them (whose refills read the next step's first
        // groups) picked by a scalar select: with the tail peeled into code of its own, the
        // register allocator gave the accumulators a rotated assignment in the loop and moved all
        // 128 of them through VGPRs at the loop exit of every step (208 accvgpr moves, C2 I8).
        for (int gb = 0; gb < G; gb += PX) {
            const bool last = gb + PX >= G;
            if (last && s + 1 < s_end) load_epi(s + 1, rin);
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
        // L2: the next step's start values after the first tail group, whose MFMAs are the last
        // reads of this step's (D = 128: the first group of the step), so they can land in the
        // same registers: issued before the tail, both sets were live at once and every step
        // copied 16 registers twice (v_mov_b64 x 16, C4).  Waits: a tail group p >= 1 has the
        // same loads younger than its slot as before ((PX - 1) slots + the start values); the
        // start values have (PX - 1) slots after them (the step-end wait below)
#pragma unroll
        for (int p = 0; p < PX; ++p) {
            group(p, gb + p, xn + (size_t)p * XGSTEP, Qbase + (size_t)(gb + p + PQ) * GSTEP);
            if (p == 0 && s + 1 < s_end) load_epi(s + 1, rin);
        }
#endif

        S8_STAMP(const unsigned long long st_c = S8_NOW(); st_k += st_c - st_a;)
#ifdef VDB_SCAN8_KLOOP_ONLY
        {  // diagnostic build (make variant): the K-loop alone, results are garbage
            int f = 0;
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int qt = 0; qt < QT; ++qt) f += imax16(aH[rt][qt]);
            if (f == 123456789) gl_s[0] = (float)f;
            if constexpr (METRIC == 1) s8_wait<RIN_YOUNGER>(rin);
            continue;
        }
#endif
        // ---- epilogue ----
        int thi[QT];
        bool qok[QT];
        float thf[QT];  // the (half-)score thresholds (INS2 / INSTHR builds)
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
            qok[qt] = qb * QB + qt * 32 + (lane & 31) < B;
            if constexpr (THC) {
                thi[qt] = thc[qt];
                thf[qt] = 0.0f;
#if VDB_S8_INS2 || VDB_S8_INSTHR
                thi[qt] = thr_of(qt, thf[qt]);
#endif
            } else {
                thi[qt] = thr_of(qt, thf[qt]);
            }
        }
        // The hot path: every tile's H maximum against the integer floor of its threshold
        uint32_t todo = 0;  // wave-uniform: bit rt * QT + qt = some lane of tile (rt, qt) passes
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
                todo |= __any(qok[qt] && imax16(aH[rt][qt]) > thi[qt]) ? 1u << (rt * QT + qt) : 0u;
        // ---- checksum: every accumulator of a row < N (a wave-uniform test per step; only the
        // last step of the corpus holds rows past N).  After the tile tests, so their ballot is not
        // held up behind it; pairwise trees, not one dependent chain per tile ----
        if (chkp) {
            if ((t0 + RT) * 32 <= N) {
#pragma unroll
                for (int qt = 0; qt < QT; ++qt) {
#pragma unroll
                    for (int rt = 0; rt < RT; ++rt) ckh[qt] += hsum16(aH[rt][qt]);
                }
            } else {
#pragma unroll
                for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                        for (int v = 0; v < 16; ++v) {
                            const int64_t row = (t0 + rt) * 32 + 8 * (v >> 2) + 4 * (lane >> 5) + (v & 3);
                            if (row < N) ckh[qt] += (uint32_t)aH[rt][qt][v];
                        }
            }
        }
        S8_STAMP(const unsigned long long st_d = S8_NOW(); st_z += st_d - st_c; st_x += (todo != 0u) + ((unsigned long long)__builtin_popcount(todo) << 20);)
        // The rare insertions: one tile at a time through ONE copy of the insertion code (the tile's
        // registers picked by a wave-uniform switch), lanes whose fp32 (half-)score H uH (+ L uL)
        // passes append; entries that find the buffer full wait in s_pend for a compaction round.
        // (With the insertion unrolled per tile, and again for the compaction rounds, the kernel
        // was 68 KB and the compiler hoisted the score conversion of all 128 accumulators out of
        // the cold blocks into every step: C6 7.6 K cycles per step in the epilogue.)
        uint32_t pmask = 0;  // wave-uniform: tiles with entries left in s_pend
        for (bool joined = false;; joined = true) {
            while (todo != 0u) {
                const int t = __builtin_amdgcn_readfirstlane(__builtin_ctz(todo));
                todo &= todo - 1u;
                i32x16 h, l;
                switch (t) {
#define S8_TILE_CASE(T_)                                                  \
    case T_:                                                              \
        if constexpr ((T_) < RT * QT) {                                   \
            h = aH[(T_) / QT][(T_) % QT];                                 \
            if constexpr (HL) l = aL[(T_) / QT][(T_) % QT];               \
        }                                                                 \
        break;
                    S8_TILE_CASE(0) S8_TILE_CASE(1) S8_TILE_CASE(2) S8_TILE_CASE(3)
                    S8_TILE_CASE(4) S8_TILE_CASE(5) S8_TILE_CASE(6) S8_TILE_CASE(7)
#undef S8_TILE_CASE
                    default: __builtin_unreachable();
                }
                static_assert(RT * QT <= 8, "tile switch covers 8 tiles");
                const int rt = t / QT, qt = t - rt * QT;
                const int ql = qt * 32 + (lane & 31);
                uint32_t gkq = gk[0];
                bool ok = qok[0];
                float thq = thf[0];
#pragma unroll
                for (int q2 = 1; q2 < QT; ++q2)
                    if (qt == q2) {
                        gkq = gk[q2];
                        ok = qok[q2];
                        thq = thf[q2];
                    }
#if VDB_S8_INS2 || VDB_S8_INSTHR
                // first round: the step's thresholds (no compaction since they were read);
                // rounds after a compaction read the raised s_thr
                float th = thq;
                if (joined) {
                    const float thr = fmaxf(s_thr[ql], key_to_float(gkq));
                    th = METRIC == 0 ? thr : 0.5f * thr;
                }
#else
                (void)thq;
                const float thr = fmaxf(s_thr[ql], key_to_float(gkq));
                const float th = METRIC == 0 ? thr : 0.5f * thr;
#endif
                const uint32_t cand = joined ? s_pend[wv][t][lane] : ok ? tile_valid16(mask, t0 + rt, N, lane) : 0u;
                const uint32_t rb = (uint32_t)((t0 + rt) * 32) + 4u * (uint32_t)(lane >> 5);
                // each lane's pass bits from 16 independent tests (no branch per register: with one
                // wave per SIMD a test-ballot-branch chain per register cost ~140 cycles, 2.9 K per
                // tile), then one round per hit of the lane with the most hits (usually one)
                float sv[16];
                uint32_t pm = 0;
#pragma unroll
                for (int v = 0; v < 16; ++v) {
                    sv[v] = HL ? fmaf((float)h[v], uH, (float)l[v] * uL) : (float)h[v] * uH;
                    pm |= (sv[v] > th ? 1u : 0u) << v;
                }
                pm &= cand;
                uint32_t left = 0;
#if VDB_S8_INS2
                // one round per register index v that some lane hits (usually one): v is
                // wave-uniform (the first hit of the first lane with hits), so the score's select
                // runs on scalar conditions, not a 16-way compare-and-select per lane
                for (;;) {
                    const unsigned long long bl = __ballot(pm != 0u);
                    if (bl == 0ull) break;
                    const int L = (int)__builtin_ctzll(bl);
                    const uint32_t pmL = (uint32_t)__builtin_amdgcn_readlane((int)pm, L);
                    const int v = __builtin_amdgcn_readfirstlane(__builtin_ctz(pmL));
                    const bool mine = (pm >> v) & 1u;
                    pm &= ~(1u << v);
                    if (mine) {
                        float a_ = sv[0];  // v uniform: scalar-masked selects, no per-lane compares
#pragma unroll
                        for (int u = 1; u < 16; ++u) a_ = v == u ? sv[u] : a_;
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
#else
                while (__any(pm != 0u)) {
                    if (pm != 0u) {
                        const int v = __builtin_ctz(pm);
                        pm &= pm - 1u;
                        float a_ = sv[0];
#pragma unroll
                        for (int u = 1; u < 16; ++u) a_ = v == u ? sv[u] : a_;
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
#endif
                if (__any(left != 0u)) {
                    s_pend[wv][t][lane] = left;
                    pmask |= 1u << t;
                }
            }
            S8_STAMP(if (!joined) { st_y += (S8_NOW() - st_c) << 20; st_f -= S8_NOW(); })
            // compaction rounds (as scan2): lockstep = a workgroup barrier per step; FLAGSYNC = a
            // wave with leftovers raises s_need and the others join at their step end
            if constexpr (!FLAGSYNC) {
                if (!__syncthreads_or(pmask != 0u)) break;
            } else {
                const bool mine = pmask != 0u;
                if (mine && lane == 0) lds_flag_st(&s_need, 1);
                if (!mine && (joined || !__builtin_amdgcn_readfirstlane(lds_flag_ld(&s_need)))) break;
                __syncthreads();  // B1
            }
            S8_STAMP(++st_y;)
            for (int q = wv; q < QB; q += NW)
                if (s_cnt[q] >= CAP)
                    compact_query<KW, CAP>(s_sc + q * CAP, s_ix + q * CAP, s_cnt + q, s_thr + q,
                                           KW == KP && qb * QB + q < B ? gthr + qb * QB + q : nullptr);
            if (FLAGSYNC && threadIdx.x == 0) lds_flag_st(&s_need, 0);
            __syncthreads();  // B2
            refresh_thr();  // the round raised s_thr
            todo = pmask;
            pmask = 0;
        }
        // the checksum's L sums (I8X3), at the end of the epilogue: the tile tests read only H,
        // so a step without passing tiles never waited for its last L MFMAs -- summing L beside
        // the H sums made every C4 step wait for the shared matrix pipe's drain (scan +7%)
        if constexpr (HL) {
            if (chkp && chk_l) {
                if ((t0 + RT) * 32 <= N) {
#pragma unroll
                    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                        for (int rt = 0; rt < RT; ++rt) ckl[qt] += hsum16(aL[rt][qt]);
                } else {
#pragma unroll
                    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                        for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                            for (int v = 0; v < 16; ++v) {
                                const int64_t row = (t0 + rt) * 32 + 8 * (v >> 2) + 4 * (lane >> 5) + (v & 3);
                                if (row < N) ckl[qt] += (uint32_t)aL[rt][qt][v];
                            }
                }
            }
        }
        // the next step's start values (RIN_YOUNGER refills issued after them; younger epilogue
        // accesses only make this wait stricter) land before the back-edge
        S8_STAMP(const unsigned long long st_g = S8_NOW(); st_f += st_g;)
        if constexpr (METRIC == 1) s8_wait<RIN_YOUNGER>(rin);
        S8_STAMP(st_q += S8_NOW() - st_g; st_e += S8_NOW() - st_c;)
    }

    // The last step's tail refilled the slots (and, global operand, the query tiles) with loads
    // nothing reads.  To the compiler those registers are free once the loop ends -- but the loads
    // are still landing: wait for them with the slots tied live until here, so no other value
    // shares their registers meanwhile.  Unconditional, so that every path to the code below --
    // including the ones the compiler cannot prove infeasible (prologue loads issued, loop not
    // entered) -- passes a vmcnt(0) (tools/vmcnt_check.py checks this on the built objects).
#pragma unroll
    for (int p = 0; p < PX; ++p) s8_wait<0>(xr[p]);
    if constexpr (!QLDS) {
#pragma unroll
        for (int p = 0; p < PQ; ++p) s8_tie(qr[p]);
    }
    if constexpr (METRIC == 1) s8_tie(rin);

    // FLAGSYNC: keep answering compaction rounds until every wave is past its last step.  A wave
    // past its last step polls (sleeping) for either: every wave done, or a round some running
    // wave called (s_need) -- then it joins that round's barriers.  (Round 4 called a round itself
    // on every poll, so once one wave of a workgroup had finished, every remaining step of the
    // others ended in two barriers: 139 rounds per wave at C4 against ~0 the lists needed.)
    if (FLAGSYNC && lane == 0) atomicAdd(&s_done, 1);
    for (; FLAGSYNC;) {
        int need = 0;
        for (;;) {
            const int done = __builtin_amdgcn_readfirstlane(lds_flag_ld(&s_done));
            need = __builtin_amdgcn_readfirstlane(lds_flag_ld(&s_need));
            if (done == NW || need) break;
            __builtin_amdgcn_s_sleep(4);
        }
        if (!need) break;  // every wave is done: nobody can call a round any more
        __syncthreads();  // B1 (the round a running wave called)
        for (int q = wv; q < QB; q += NW)
            if (s_cnt[q] >= CAP)
                compact_query<KW, CAP>(s_sc + q * CAP, s_ix + q * CAP, s_cnt + q, s_thr + q,
                                       KW == KP && qb * QB + q < B ? gthr + qb * QB + q : nullptr);
        if (threadIdx.x == 0) lds_flag_st(&s_need, 0);
        __syncthreads();  // B2
    }

    // the checksum's partial sums: lane halves of a query column, then the waves through LDS,
    // one word per (plane, workgroup, query) -- no atomics on global memory, summed by the finish
    if (chkp) {
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
            const uint32_t h = ckh[qt] + (uint32_t)__shfl_xor((int)ckh[qt], 32, 64);
            const uint32_t l = ckl[qt] + (uint32_t)__shfl_xor((int)ckl[qt], 32, 64);
            if (lane < 32) {
                atomicAdd(&s_chk[0][qt * 32 + lane], h);
                if constexpr (HL) atomicAdd(&s_chk[HL ? 1 : 0][qt * 32 + lane], l);
            }
        }
    }
    // ---- flush: entries above the shared bound -> global per-query lists ----
    __syncthreads();
    if (chkp) {
        const int nwg8 = (int)(gridDim.x / (unsigned)n_qb);
        for (int i = threadIdx.x; i < (HL ? 2 : 1) * QB; i += 64 * NW) {
            const int pl = i / QB, q = i - pl * QB;
            chkp[((size_t)pl * chk_ld + (size_t)qb * QB + q) * nwg8 + wg] = s_chk[pl][q];
        }
    }
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
#ifdef VDB_STAMP8
    {
        const int w = blockIdx.x * NW + wv;
        if (lane == 0 && w < (1 << 16)) {
            const unsigned long long v[12] = {S8_NOW() - st_t0, st_w, st_k, st_e, st_n, st_r0, st_x, st_y, st_z,
                                              __builtin_amdgcn_s_memrealtime(), st_q, st_f};
#pragma unroll
            for (int i = 0; i < 12; ++i) g_scan8_stamps[w][i] = v[i];
        }
    }
#endif
}

// ---- launch templates ----
template <int P, int M, int QT, int PX, int KP, int CAP, bool NT, bool QL, bool FS, int GC, int RT_ = scan8_rt(P, M),
          int KW = KP>
static hipError_t scan8_launch_g(const float* Xq, const float* rinit, const uint32_t* mask, const float* Qq,
                                 const float* lsl, const float* qscal, int G, int64_t N, int B, int n_qblocks,
                                 int64_t n_steps, int n_wg, int spw, float* gl_s, uint32_t* gl_i, uint32_t* gl_cnt,
                                 int64_t gl_cap, uint32_t* gthr, const int* gate,
                                 uint32_t* chkp, int chk_ld, int chk_l, hipStream_t st) {
    auto k = scan8_kernel<P, M, QT, PX, KP, CAP, NT, QL, FS, GC, RT_, KW>;
    const size_t lds = QL ? (size_t)G * Planes8<P>::QPL * QT * 1024 : 0;
    if (QL) {
        static std::atomic<size_t> lds_set{0};
        size_t cur = lds_set.load();
        while (lds > cur) {
            hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
            if (lds_set.compare_exchange_weak(cur, lds)) break;
        }
    }
    const int n_wg8 = (n_wg + 7) / 8 * 8;
    hipLaunchKernelGGL(k, dim3(n_wg8 * n_qblocks), dim3(64 * scan8_nw(P, M, QT)), lds, st, Xq, rinit, mask, Qq, lsl, qscal, G, N, B,
                       n_steps, spw, n_qblocks, gl_s, gl_i, gl_cnt, gl_cap, gthr, gate, chkp, chk_ld, chk_l);
    return hipGetLastError();
}

template <int P, int M, int QT, int PX, int KP, int CAP, bool NT, bool QL, bool FS, int KW = KP,
          int RT_ = scan8_rt(P, M)>
static hipError_t scan8_launch(const float* Xq, const float* rinit, const uint32_t* mask, const float* Qq,
                               const float* lsl, const float* qscal, int G, int64_t N, int B, int n_qblocks,
                               int64_t n_steps, int n_wg, int spw, float* gl_s, uint32_t* gl_i, uint32_t* gl_cnt,
                               int64_t gl_cap, uint32_t* gthr, const int* gate,
                               uint32_t* chkp, int chk_ld, int chk_l, hipStream_t st) {
    if constexpr (QL) {
        if (G == 4)  // D = 128: the group loop unrolls, and the whole next step is in flight
            return scan8_launch_g<P, M, QT, 4, KP, CAP, NT, QL, FS, 4, RT_, KW>(Xq, rinit, mask, Qq, lsl, qscal, G, N, B,
                                                                        n_qblocks, n_steps, n_wg, spw, gl_s, gl_i,
                                                                        gl_cnt, gl_cap, gthr, gate,
                                                                        chkp, chk_ld, chk_l, st);
    }
    // the step loop takes the groups PX at a time: Dp / 32 groups is only even (D = 192: 6), so
    // where PX does not divide them the 2-deep variant runs (4 deep, the tail's refills would read
    // the next row tile's groups into this one's scores)
    if constexpr (PX != 2) {
        if (G % PX != 0)
            return scan8_launch_g<P, M, QT, 2, KP, CAP, NT, QL, FS, 0, RT_, KW>(
                Xq, rinit, mask, Qq, lsl, qscal, G, N, B, n_qblocks, n_steps, n_wg, spw, gl_s, gl_i, gl_cnt, gl_cap,
                gthr, gate, chkp, chk_ld, chk_l, st);
    }
    return scan8_launch_g<P, M, QT, PX, KP, CAP, NT, QL, FS, 0, RT_, KW>(Xq, rinit, mask, Qq, lsl, qscal, G, N, B, n_qblocks,
                                                                n_steps, n_wg, spw, gl_s, gl_i, gl_cnt, gl_cap, gthr,
                                                                gate, chkp, chk_ld, chk_l, st);
}

// The query block in LDS takes the query operand off each wave's vector-memory path (from L2,
// 64 queries x 32 dims per plane and group beside the corpus tiles).  It fits when the block
// (64 queries x D bytes per plane; I8 reads qh alone) plus the static LDS (64 queries x CAP x
// 8 B of lists, s_pend 8 KiB, counters) is within the CU's 160 KiB: C3 (D = 1536, I8, KP = 256
// with CAP 96): 96 + 56.5 KiB.  `small` keeps the round-3 rule (block <= 32 KiB: short rows).
inline int scan8_qpl(int prec) { return prec == PREC_I8X3 || prec == PREC_I8Q ? 2 : 1; }
inline int scan8_cap(int KP, bool ql) { return KP == 128 ? 192 : KP == 256 ? (ql ? 96 : 128) : 128; }  // as S8_KP
inline bool scan8_qlds(int G8, int KP, int prec, int metric, bool small) {
    const size_t q = (size_t)G8 * scan8_qpl(prec) * 2 * 1024;
    if (small) return q <= 32 * 1024;
    // lists, s_pend of this shape's waves (the 8-wave I8X3 L2 shape: 16 KiB; counted at 8 waves for
    // every shape, C3's 96 KiB query block stopped fitting beside its 48 KiB of lists at the end of
    // round 4), counters and the checksum's sums
    const size_t lists = (size_t)64 * scan8_cap(KP, true) * 8 + (size_t)scan8_nw(prec, metric) * 2048 + 1536;
    return lists + q <= 160 * 1024;
}


#define S8_UNIT_PARAMS                                                                                             \
    int KP, const float *Xq, const float *rinit, const uint32_t *mask, const float *Qq, const float *lsl,          \
        const float *qscal, int G, int64_t N, int B, int n_qblocks, int64_t n_steps, int n_wg, int spw,           \
        float *gl_s, uint32_t *gl_i, uint32_t *gl_cnt, int64_t gl_cap, uint32_t *gthr, bool nt, bool ql, bool fs,  \
        const int *gate, uint32_t *chkp, int chk_ld, int chk_l,                                                     \
        hipStream_t st
#define S8_ARGS \
    Xq, rinit, mask, Qq, lsl, qscal, G, N, B, n_qblocks, n_steps, n_wg, spw, gl_s, gl_i, gl_cnt, gl_cap, gthr, gate, \
        chkp, chk_ld, chk_l, st
#define S8_ONE(P, M, KPV, QTV, PXV, CAPV, NTV, QLV, FSV, KWV)   \
    if (KP == KPV && nt == NTV && ql == QLV && fs == FSV)        \
        return scan8_launch<P, M, QTV, PXV, KPV, CAPV, NTV, QLV, FSV, KWV>(S8_ARGS);
// KP = 256 keeps 64-query blocks: a workgroup keeps its best KW = 64 per query (LDS 64 KiB, 48
// with the query block in LDS beside it; the drop bound -> gthr, vdb_scan2_kernel.h), so a
// 64-query batch reads the corpus once
#define S8_KP(P, M, PXV, NTV, QLV, FSV)               \
    S8_ONE(P, M, 32, 2, PXV, 128, NTV, QLV, FSV, 32)   \
    S8_ONE(P, M, 64, 2, PXV, 128, NTV, QLV, FSV, 64)   \
    S8_ONE(P, M, 128, 2, PXV, 192, NTV, QLV, FSV, 128) \
    S8_ONE(P, M, 256, 2, PXV, (QLV ? 96 : 128), NTV, QLV, FSV, 64)
// one query block with the query block in LDS: the corpus loads non-temporal too (VDB_S8_NTQL)
#if VDB_S8_NTQL
#define S8_KP_NTQL(P, M, PXL) S8_KP(P, M, PXL, true, true, true)
#else
#define S8_KP_NTQL(P, M, PXL)
#endif
#define S8_MODES(P, M, PXV, PXL)                                               \
    S8_KP(P, M, PXV, false, false, false) S8_KP(P, M, PXV, true, false, false) \
    S8_KP(P, M, PXL, false, true, false) S8_KP(P, M, PXL, false, true, true)   \
    S8_KP(P, M, PXV, false, false, true) S8_KP(P, M, PXV, true, false, true)   \
    S8_KP_NTQL(P, M, PXL)
#define S8_UNIT(NAME, P, M, PXV, PXL)  \
    hipError_t NAME(S8_UNIT_PARAMS) {  \
        S8_MODES(P, M, PXV, PXL)       \
        return hipErrorInvalidValue;   \
    }
hipError_t launch_scan8_i1c(S8_UNIT_PARAMS);
hipError_t launch_scan8_i1l(S8_UNIT_PARAMS);
hipError_t launch_scan8_i3c(S8_UNIT_PARAMS);
hipError_t launch_scan8_i3l(S8_UNIT_PARAMS);
hipError_t launch_scan8_iqc(S8_UNIT_PARAMS);
hipError_t launch_scan8_iql(S8_UNIT_PARAMS);

}  // namespace vdb
