// vdb_scan8w.hip — the int8 candidate pass for short rows and large batches (round 6): the
// "wide" shape.  Used for D <= 128 (4 groups of 32 dims) and B > 256 (C4: 10M x 128 L2 top-100,
// B = 512, and every rank of its 8-way row-sharded run).
//
// Why a second shape.  scan8_kernel (vdb_scan8_kernel.h) gives each workgroup ONE 64-query block
// and streams the corpus through registers, so C4's 8 query blocks read every row 8 times (from
// L2 when they stay close), with the query block in LDS beside per-query candidate lists.  A
// build whose steps end after the K-loop ran C4's scan in 0.94 ms against 1.61 ms for the real
// kernel and 0.52 ms of MFMA time (profiles/r06_ab): the K-loop alone waited on its L2 stream,
// and the epilogue (tile tests, LDS lists, compaction flags) took the rest.
//
// Here one workgroup of 8 waves holds ALL of up to 512 queries, one 64-query block per wave, and
// each wave keeps its block's int8 tiles in REGISTERS for the whole launch (D = 128: 4 groups x 2
// query tiles x 2 planes = 64 VGPRs).  The corpus is read from HBM exactly once: row tiles are
// staged into a two-slot LDS ring by LDS-DMA (global_load_lds_dwordx4, no VGPR destination), every
// wave reads each staged tile's A operand from LDS (4 ds_read_b128 per tile), and the slots turn
// over behind one workgroup barrier per stage of NTILE row tiles (16 for one corpus plane, 8 for
// two: 64 KiB of corpus per slot).  The loads of stage m + 1 are issued right after stage m's
// barrier, so a whole stage of MFMA work (NTILE x 16 MFMAs per wave) covers their latency.
//
// No LDS candidate lists: the shared bound is the pilot's (gthr, fixed for the launch), so a row
// whose (half-)score passes it goes straight to its query's global list.  Each (workgroup, query)
// owns a fixed segment of W8_CH slots of that list (no global atomics): the position comes from
// an LDS counter of the wave that owns the query; the segment counts go to seg_cnt [B][n_seg]
// and the finish reads the segments (vdb_exact.hip, seg mode).  A segment that would overflow
// makes the finish send its query to the exact path (correct, slow).  Row tiles are dealt to the
// workgroups one at a time (tile t -> workgroup t mod n_seg), so a run of similar rows spreads over
// all segments: with C4's pilot bound ~2 entries per segment and query are expected.
//
// Certificate invariant (vdb_exact.hip finish_kernel): every row not in its query's list scored
// (this arithmetic) <= the final shared bound (gthr, the pilot's), so acut = max(a_KP, T) holds.
// The checksum (vdb_scan8.hip) is unchanged: per lane the sums of every H (and L) accumulator of
// the rows < N this workgroup scored, one word per (plane, query, workgroup).
#include "vdb_scan8_kernel.h"

namespace vdb {

// waves per workgroup and query tiles (32 queries) per wave: 8 x 2 (two waves per SIMD, 64
// queries each) by default; 16 x 1 (four per SIMD) an A/B build
#ifndef VDB_W8_NW
#define VDB_W8_NW 8
#endif
#ifndef VDB_W8_QT
#define VDB_W8_QT 2
#endif
// A/B build knobs: VDB_W8_PF 1 = the next tile's operands read from LDS before this tile's
// MFMAs; VDB_W8_STAGGER n = the second wave of each SIMD starts every stage ~64 n cycles late
#ifndef VDB_W8_PF
#define VDB_W8_PF 0
#endif
#ifndef VDB_W8_STAGGER
#define VDB_W8_STAGGER 0
#endif
// VDB_W8_HFIRST 1 (default): a tile's H products (the tile tests' operand) issued before its L
// products, so the tile tests run under the wave's own L MFMAs (C4 scan -1..2%, r06_wide7)
#ifndef VDB_W8_HFIRST
#define VDB_W8_HFIRST 1
#endif
constexpr int W8_NW = VDB_W8_NW;
constexpr int W8_QT = VDB_W8_QT;
constexpr int W8_G = 4;    // 32-dim groups (Dp = 128)
constexpr int W8_QW = W8_QT * 32;    // queries per wave
constexpr int W8_QB = W8_NW * W8_QW;  // queries per workgroup
static_assert(W8_QB == 512, "512 queries per workgroup");

// SM: the small stage (8 one-plane row tiles, 32 KiB per slot) of batches of <= 256 queries: the
// pass then leaves LDS for the finish's small form beside it (vdb_exact.hip FIN_CAP_SMALL)
template <int PREC, bool SM = false>
#ifndef VDB_W8_SM_NTILE
#define VDB_W8_SM_NTILE 8
#endif
__host__ __device__ constexpr int w8_ntile() { return Planes8<PREC>::XPL == 2 ? 8 : SM ? VDB_W8_SM_NTILE : 16; }
template <int PREC, int METRIC, bool SM = false>
__host__ __device__ constexpr size_t w8_slot_bytes() {
    return (size_t)w8_ntile<PREC, SM>() * W8_G * Planes8<PREC>::XPL * 1024 + (METRIC == 1 ? (size_t)w8_ntile<PREC, SM>() * 128 : 0);
}
template <int PREC, int METRIC, bool SM = false>
__host__ __device__ constexpr size_t w8_lds_bytes() { return 2 * w8_slot_bytes<PREC, METRIC, SM>() + (size_t)3 * W8_QB * 4; }

// the LDS byte address of a __shared__ object (the LDS-DMA destination base is an address, M0)
__device__ __forceinline__ uint32_t w8_lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

// One LDS-DMA load: lane l's 16 bytes at gsrc go to LDS byte lds + 16 l.  M0 is compiler-reserved,
// so it is saved and restored inside the same statement; the asm is invisible to hipcc's wait
// counting: the stage barrier below waits vmcnt(0) for it.
template <bool NT>
__device__ __forceinline__ void w8_glds(const void* gsrc, uint32_t lds) {
    uint32_t keep;
    if constexpr (NT)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(gsrc), "s"(lds) : "memory");
    else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(gsrc), "s"(lds) : "memory");
}

template <int PREC, int METRIC, bool NT, bool SM>
__global__ void __launch_bounds__(64 * W8_NW, 1)
scan8w_kernel(const float* __restrict__ Xq, const int* __restrict__ rs8, const uint32_t* __restrict__ mask,
              const float* __restrict__ Qq, const float* __restrict__ lsl, const float* __restrict__ qscal, int64_t N,
              int B, int Bp, float* __restrict__ gl_s, uint32_t* __restrict__ gl_i, int64_t gl_cap,
              uint32_t* __restrict__ seg_cnt, const uint32_t* __restrict__ gthr, uint32_t* __restrict__ chkp, int chk_ld,
              int chk_l, int rw) {
    constexpr int G = W8_G, QT = W8_QT, NW = W8_NW;
    constexpr int XPL = Planes8<PREC>::XPL, QPL = Planes8<PREC>::QPL;
    constexpr bool HL = Planes8<PREC>::L;
    constexpr int NTILE = METRIC == 1 && SM ? 8 : w8_ntile<PREC, SM>();  // (L2: the start values load 8 tiles per wave)
    static_assert(METRIC == 0 || NTILE % 8 == 0, "L2 start values: 8 row tiles per loading wave");
    constexpr size_t TILE_B = (size_t)G * XPL * 1024;
    constexpr size_t CORP_B = NTILE * TILE_B;
    constexpr size_t SLOT_B = w8_slot_bytes<PREC, METRIC, SM>();
    constexpr size_t GSTEP = 8 * BLOCK_FLOATS, PLANE = 4 * BLOCK_FLOATS;
    constexpr int QW = W8_QW;
    constexpr int LPW = XPL * NTILE * G / NW;  // corpus loads per wave and stage
    static_assert(XPL * NTILE * G == LPW * NW, "corpus loads spread evenly over the waves");
    extern __shared__ __attribute__((aligned(16))) char s_dyn[];

    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int w = blockIdx.x, n_seg = gridDim.x;
    // rw waves per 64-query block (a small batch: the stage's tiles split over them, tile i to
    // wave i mod rw of the block; rw = 1 for C4's 512 queries)
    const int n_qb = NW / rw, qbl = wv % n_qb, rl = wv / n_qb;
    const int q0 = (blockIdx.y * n_qb + qbl) * QW;  // this wave's queries q0 .. q0 + QW - 1
    const bool active = q0 < Bp;                 // (wave-uniform: a block past the padded batch only loads)
    int* s_seg = (int*)(s_dyn + 2 * SLOT_B);     // rw > 1: [n_qb * QW] entries per query of the workgroup
    uint32_t* s_ck = (uint32_t*)(s_seg + W8_QB);  //          and its checksum words [2][n_qb * QW]
    if (rw > 1)
        for (int i = threadIdx.x; i < 3 * W8_QB; i += 64 * NW) s_seg[i] = 0;
    const int64_t T = (N + 31) >> 5;
    const int64_t my_tiles = T > w ? (T - 1 - w) / n_seg + 1 : 0;
    const int64_t n_stages = (my_tiles + NTILE - 1) / NTILE;
    const uint32_t ring = w8_lds_addr(s_dyn);

    // this workgroup's entries per query tile of the lane, in registers: a query tile belongs to
    // one wave, so lanes l and l + 32 (the tile's two row halves) count it together (no LDS
    // atomic round trip on the insertion path)
    int cnt[QT];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) cnt[qt] = 0;

    // This wave's share of stage m's LDS-DMA loads into slot sl: LPW of the stage's 64 corpus
    // blocks (1 KiB each: row tile, group, plane) and, L2, waves 0 .. NTILE / 8 - 1 one 1 KiB piece
    // of the batch's integer start values each (8 row tiles x 128 B, a per-lane source address)
    auto issue = [&](int64_t m, int sl) {
        const uint32_t sbase = ring + (uint32_t)(sl * SLOT_B);
#pragma unroll
        for (int u = 0; u < LPW; ++u) {
            const int j = wv * LPW + u;  // (tile, group, plane) block j of the stage
            const int i = j / (G * XPL), g = (j / XPL) % G, pl = j % XPL;
            const int64_t t = (m * NTILE + i) * n_seg + w;
            if (t < T)
                w8_glds<NT>(Xq + corpus_block((uint64_t)t, g, pl, G) + lane * 4, sbase + (uint32_t)(j * 1024));
        }
        if constexpr (METRIC == 1) {
            if (wv < NTILE / 8) {
                const int i = wv * 8 + (lane >> 3);
                int64_t t = (m * NTILE + i) * n_seg + w;
                if (t >= T) t = 0;  // (a tile no wave scores: any valid source)
                w8_glds<NT>(rs8 + t * 32 + (lane & 7) * 4, sbase + (uint32_t)(CORP_B + wv * 1024));
            }
        }
    };

    // the query block's tiles, whole, in registers; per query tile the pilot's bound (fixed for
    // the launch) as the (half-)score threshold and its integer floor for the tile tests
    const float uH = qscal[0], uL = qscal[1], invU = qscal[2];
    f32x4 qr[G][QT][QPL];
    float thf[QT];
    int thc[QT];
    uint32_t ckh[QT], ckl[QT];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
        const int q = q0 + qt * 32 + (lane & 31);
        const bool ok = active && q < B;
        const float th = ok ? key_to_float(gthr[q]) : INFINITY;
        thf[qt] = METRIC == 0 ? th : 0.5f * th;
        thc[qt] = ok ? h_floor(thf[qt], lsl[q], invU) : INT_MAX;
        ckh[qt] = ckl[qt] = 0u;
    }
    if (active) {
        const float* qs = Qq + s2_blk((uint64_t)(q0 / 32), 0, G + QG_EXTRA) + lane * 4;
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                for (int pl = 0; pl < QPL; ++pl) qr[g][qt][pl] = *(const f32x4*)(qs + g * GSTEP + pl * PLANE + qt * BLOCK_FLOATS);
    }
    if (n_stages > 0) issue(0, 0);

    for (int64_t m = 0; m < n_stages; ++m) {
        // this wave's loads of stage m have landed (vmcnt 0: nothing younger is in flight yet);
        // after the barrier every wave's have, and every wave is done with stage m - 1, whose
        // slot stage m + 1 now refills
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (m + 1 < n_stages) issue(m + 1, (int)((m + 1) & 1));
        if (!active) continue;
#if VDB_W8_STAGGER > 0
        // the waves sharing a SIMD (w, w + 4, ...: a workgroup's waves go to the SIMDs in a fixed
        // cyclic order) start the stage a fraction of a tile apart, so one's epilogue runs under
        // the other's MFMAs instead of all of them leaving the matrix pipe idle together
        for (int z = 0; z < (wv >> 2) * VDB_W8_STAGGER / (NW >> 2); ++z) __builtin_amdgcn_s_sleep(1);
#endif
        const char* slot = s_dyn + (size_t)(m & 1) * SLOT_B;
        const int n_here = (int)min<int64_t>(NTILE, my_tiles - m * NTILE);  // this stage's tiles
        // a tile's operands from the slot: the A blocks and (L2) the rows' integer start values
        // (lane half h holds rows 32 t + 8 a + 4 h + b of its accumulator registers 4 a + b)
        auto ld_tile = [&](int i, f32x4 (&x)[G][1][XPL], i32x4 (&r)[4]) {
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int pl = 0; pl < XPL; ++pl)
                    x[g][0][pl] = *(const f32x4*)(slot + (size_t)i * TILE_B + (size_t)((g * XPL + pl) * 1024) + lane * 16);
            if constexpr (METRIC == 1) {
#pragma unroll
                for (int a = 0; a < 4; ++a)
                    r[a] = *(const i32x4*)(slot + CORP_B + (size_t)i * 128 + (size_t)(8 * a + 4 * (lane >> 5)) * 4);
            }
        };
#if VDB_W8_PF
        f32x4 xr[G][1][XPL];
        i32x4 rr[4];
        ld_tile(0, xr, rr);
#endif
        for (int i = rl; i < n_here; i += rw) {
            const int64_t t = (m * NTILE + i) * n_seg + w;
#if VDB_W8_PF
            f32x4 xn[G][1][XPL];
            i32x4 rn[4];
#else
            f32x4 xr[G][1][XPL];
            i32x4 rr[4];
            ld_tile(i, xr, rr);
#endif
            i32x16 aH[1][QT], aL[1][QT];
            {
                i32x16 init;
#pragma unroll
                for (int v = 0; v < 16; ++v) init[v] = METRIC == 1 ? rr[v >> 2][v & 3] : 0;
#pragma unroll
                for (int qt = 0; qt < QT; ++qt) {
                    aH[0][qt] = init;
#pragma unroll
                    for (int v = 0; v < 16; ++v) aL[0][qt][v] = 0;
                }
            }
#if VDB_W8_HFIRST
            // every H product of the tile first, then the L ones: the tile tests read H alone, so
            // they run while the wave's own L MFMAs still execute
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int qt = 0; qt < QT; ++qt)
                    aH[0][qt] = __builtin_amdgcn_mfma_i32_32x32x32_i8(__builtin_bit_cast(i32x4, xr[g][0][0]),
                                                                      __builtin_bit_cast(i32x4, qr[g][qt][0]), aH[0][qt], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);  // (the scheduler would interleave them again)
            if constexpr (HL) {
#pragma unroll
                for (int g = 0; g < G; ++g)
#pragma unroll
                    for (int qt = 0; qt < QT; ++qt) {
                        aL[0][qt] = __builtin_amdgcn_mfma_i32_32x32x32_i8(__builtin_bit_cast(i32x4, xr[g][0][0]),
                                                                          __builtin_bit_cast(i32x4, qr[g][qt][QPL - 1]), aL[0][qt], 0, 0, 0);
                        if constexpr (PREC == PREC_I8X3)
                            aL[0][qt] = __builtin_amdgcn_mfma_i32_32x32x32_i8(__builtin_bit_cast(i32x4, xr[g][0][XPL - 1]),
                                                                              __builtin_bit_cast(i32x4, qr[g][qt][0]), aL[0][qt], 0, 0, 0);
                    }
            }
            if (false)
#endif
            group_mfma8<PREC, 1, QT>(xr[0], qr[0], aH, aL);
#if VDB_W8_PF
            // the next tile's operands, read after this tile's first MFMAs issued: their LDS
            // latency runs under this tile's MFMAs (read before them, hipcc's loop-header wait
            // for the operands in flight waited for these too: lgkmcnt(0) before the first MFMA)
            __builtin_amdgcn_sched_barrier(0);
            if (i + 1 < n_here) ld_tile(i + 1, xn, rn);
            __builtin_amdgcn_sched_barrier(0);
#endif
#pragma unroll
            for (int g = 1; g < G; ++g)
                if (!VDB_W8_HFIRST) group_mfma8<PREC, 1, QT>(xr[g], qr[g], aH, aL);
#if VDB_W8_PF
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int pl = 0; pl < XPL; ++pl) xr[g][0][pl] = xn[g][0][pl];
#pragma unroll
            for (int a = 0; a < 4; ++a) rr[a] = rn[a];
#endif

#ifdef VDB_SCAN8W_KLOOP_ONLY
            {  // diagnostic build (make wvariant): the K-loop alone, results are garbage
                int f = 0;
#pragma unroll
                for (int qt = 0; qt < QT; ++qt) f += imax16(aH[0][qt]) + (HL ? imax16(aL[0][qt]) : 0);
                if (f == 123456789) gl_s[0] = (float)f;
                continue;
            }
#endif
            // ---- epilogue: the tile tests (H only, minus the L term's slack), the checksum ----
            uint32_t todo = 0;
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
                todo |= __builtin_amdgcn_ballot_w64(imax16(aH[0][qt]) > thc[qt]) != 0ull ? 1u << qt : 0u;
            if (chkp) {
                if ((t + 1) * 32 <= N) {
#pragma unroll
                    for (int qt = 0; qt < QT; ++qt) ckh[qt] += hsum16(aH[0][qt]);
                    if constexpr (HL) {
                        if (chk_l) {
#pragma unroll
                            for (int qt = 0; qt < QT; ++qt) ckl[qt] += hsum16(aL[0][qt]);
                        }
                    }
                } else {
#pragma unroll
                    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                        for (int v = 0; v < 16; ++v) {
                            const int64_t row = t * 32 + 8 * (v >> 2) + 4 * (lane >> 5) + (v & 3);
                            if (row < N) {
                                ckh[qt] += (uint32_t)aH[0][qt][v];
                                if (HL && chk_l) ckl[qt] += (uint32_t)aL[0][qt][v];
                            }
                        }
                }
            }
#ifdef VDB_SCAN8W_NOINS
            if (todo == 0xdeadu) gl_s[1] = 0.0f;  // diagnostic build: tile tests without insertions
            todo = 0;
#endif
            // ---- the rare insertions: straight into this (workgroup, query) segment ----
            while (todo != 0u) {
                const int qt = __builtin_amdgcn_readfirstlane(__builtin_ctz(todo));
                todo &= todo - 1u;
                const i32x16 h = qt == 0 ? aH[0][0] : aH[0][QT - 1];
                i32x16 l;
                if constexpr (HL) l = qt == 0 ? aL[0][0] : aL[0][QT - 1];
                const int ql = qt * 32 + (lane & 31);
                const int qg = q0 + ql;
                const float th = qt == 0 ? thf[0] : thf[QT - 1];
                const uint32_t cand = qg < B ? tile_valid16(mask, t, N, lane) : 0u;
                float sv[16];
                uint32_t pm = 0;
#pragma unroll
                for (int v = 0; v < 16; ++v) {
                    sv[v] = HL ? fmaf((float)h[v], uH, (float)l[v] * uL) : (float)h[v] * uH;
                    pm |= (sv[v] > th ? 1u : 0u) << v;
                }
                pm &= cand;
                int pos;
                if (rw == 1) {
                    const int np = __builtin_popcount(pm);
                    const int np_hi = __shfl_xor(np, 32, 64);  // (the other row half's)
                    pos = (qt == 0 ? cnt[0] : cnt[QT - 1]) + (lane >= 32 ? np_hi : 0);
                    if (qt == 0) cnt[0] += np + np_hi;
                    else cnt[QT - 1] += np + np_hi;
                } else {  // (the block's rw waves share the segment)
                    pos = pm != 0u ? atomicAdd(&s_seg[qbl * QW + ql], __builtin_popcount(pm)) : 0;
                }
                const uint32_t rb = (uint32_t)(t * 32) + 4u * (uint32_t)(lane >> 5);
                float* ls = gl_s + (size_t)qg * gl_cap + (size_t)w * W8_CH;
                uint32_t* li = gl_i + (size_t)qg * gl_cap + (size_t)w * W8_CH;
                while (pm != 0u) {
                    const int v = __builtin_ctz(pm);
                    pm &= pm - 1u;
                    float a_ = sv[0];
#pragma unroll
                    for (int u = 1; u < 16; ++u) a_ = v == u ? sv[u] : a_;
                    if (pos < W8_CH) {
                        ls[pos] = METRIC == 0 ? a_ : 2.0f * a_;
                        li[pos] = rb + (uint32_t)((v & 3) + 8 * (v >> 2));
                    }
                    ++pos;
                }
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (rw > 1) {
        // the rw waves' checksum partial sums of each query summed in LDS, then one word per
        // (plane, query, workgroup), and the segment counts
        if (active && chkp) {
#pragma unroll
            for (int qt = 0; qt < QT; ++qt) {
                const uint32_t hsum = ckh[qt] + (uint32_t)__shfl_xor((int)ckh[qt], 32, 64);
                const uint32_t lsum = ckl[qt] + (uint32_t)__shfl_xor((int)ckl[qt], 32, 64);
                if (lane < 32) {
                    atomicAdd(&s_ck[qbl * QW + qt * 32 + lane], hsum);
                    if (HL && chk_l) atomicAdd(&s_ck[W8_QB + qbl * QW + qt * 32 + lane], lsum);
                }
            }
        }
        __syncthreads();
        for (int i = threadIdx.x; i < n_qb * QW; i += 64 * NW) {
            const int q = blockIdx.y * n_qb * QW + i;
            if (q >= B) continue;
            seg_cnt[(size_t)q * n_seg + w] = (uint32_t)s_seg[i];
            if (chkp) {
                chkp[(size_t)q * n_seg + w] = s_ck[i];
                if (HL && chk_l) chkp[((size_t)chk_ld + q) * n_seg + w] = s_ck[W8_QB + i];
            }
        }
        return;
    }
    if (!active) return;
    // this workgroup's entries per query (the finish's segment counts; > W8_CH = overflowed)
#pragma unroll
    for (int qt = 0; qt < QT; ++qt)
        if (lane < 32 && q0 + qt * 32 + lane < B) seg_cnt[(size_t)(q0 + qt * 32 + lane) * n_seg + w] = (uint32_t)cnt[qt];
    // the checksum's partial sums: the tile's two row halves (lanes l, l + 32), one word per
    // (plane, query, workgroup)
    if (chkp) {
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
            const uint32_t hsum = ckh[qt] + (uint32_t)__shfl_xor((int)ckh[qt], 32, 64);
            const uint32_t lsum = ckl[qt] + (uint32_t)__shfl_xor((int)ckl[qt], 32, 64);
            const int q = q0 + qt * 32 + lane;
            if (lane < 32 && q < B) {
                chkp[(size_t)q * n_seg + w] = hsum;
                if (HL && chk_l) chkp[((size_t)chk_ld + q) * n_seg + w] = lsum;
            }
        }
    }
}

bool scan8w_ok(int G8, int B) { return G8 == W8_G && B >= 1; }
// waves per 64-query block: the whole workgroup for a batch of <= 64 queries, 4 / 2 for <= 128 /
// <= 256, one for C4's 512
int scan8w_rw(int B) { return B <= 64 ? 8 : B <= 128 ? 4 : B <= 256 ? 2 : 1; }
int scan8w_qblocks(int B) {
    const int per_wg = W8_QB / scan8w_rw(B);
    return (B + per_wg - 1) / per_wg;
}

template <int P, int M, bool NT, bool SM>
static hipError_t scan8w_launch(const float* Xq, const int* rs8, const uint32_t* mask, const float* Qq, const float* lsl,
                                const float* qscal, int64_t N, int B, int Bp, int n_seg, float* gl_s, uint32_t* gl_i,
                                int64_t gl_cap, uint32_t* seg_cnt, const uint32_t* gthr, uint32_t* chkp, int chk_ld,
                                int chk_l, hipStream_t st) {
    auto k = scan8w_kernel<P, M, NT, SM>;
    constexpr size_t lds = w8_lds_bytes<P, M, SM>();
    static_assert(lds <= 160 * 1024, "LDS");
    static std::atomic<bool> lds_set{false};
    if (!lds_set.load()) {
        const hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        lds_set = true;
    }
    hipLaunchKernelGGL(k, dim3((unsigned)n_seg, (unsigned)scan8w_qblocks(B)), dim3(64 * W8_NW), lds, st, Xq, rs8, mask, Qq,
                       lsl, qscal, N, B, Bp, gl_s, gl_i, gl_cap, seg_cnt, gthr, chkp, chk_ld, chk_l, scan8w_rw(B));
    return hipGetLastError();
}

hipError_t launch_scan8w(int prec, int metric, const float* Xq, const int* rs8, const uint32_t* mask, const float* Qq,
                         const float* lsl, const float* qscal, int G8, int64_t N, int B, int Bp, int n_seg,
                         float* gl_s, uint32_t* gl_i, int64_t gl_cap, uint32_t* seg_cnt, const uint32_t* gthr,
                         uint32_t* chkp, int chk_ld, int chk_l, hipStream_t st) {
    if (!scan8w_ok(G8, B) || n_seg <= 0 || gl_cap != (int64_t)n_seg * W8_CH || (metric == 1 && !rs8))
        return hipErrorInvalidValue;
    // the corpus is read once per query block: non-temporal with one (C4), default policy with
    // several (they share each tile through the XCD's L2)
    const bool nt = scan8w_qblocks(B) == 1;
    const bool sm = scan8w_rw(B) > 1;
#define W8_CASE(P, M)                                                                                                 \
    if (prec == P && metric == M) {                                                                                   \
        if (sm)                                                                                                       \
            return nt ? scan8w_launch<P, M, true, true>(Xq, rs8, mask, Qq, lsl, qscal, N, B, Bp, n_seg, gl_s, gl_i,   \
                                                        gl_cap, seg_cnt, gthr, chkp, chk_ld, chk_l, st)              \
                      : scan8w_launch<P, M, false, true>(Xq, rs8, mask, Qq, lsl, qscal, N, B, Bp, n_seg, gl_s, gl_i,  \
                                                         gl_cap, seg_cnt, gthr, chkp, chk_ld, chk_l, st);            \
        return nt ? scan8w_launch<P, M, true, false>(Xq, rs8, mask, Qq, lsl, qscal, N, B, Bp, n_seg, gl_s, gl_i,      \
                                                     gl_cap, seg_cnt, gthr, chkp, chk_ld, chk_l, st)                 \
                  : scan8w_launch<P, M, false, false>(Xq, rs8, mask, Qq, lsl, qscal, N, B, Bp, n_seg, gl_s, gl_i,     \
                                                      gl_cap, seg_cnt, gthr, chkp, chk_ld, chk_l, st);               \
    }
    W8_CASE(PREC_I8Q, 1) W8_CASE(PREC_I8X3, 1) W8_CASE(PREC_I8, 1)
    W8_CASE(PREC_I8Q, 0) W8_CASE(PREC_I8X3, 0) W8_CASE(PREC_I8, 0)
#undef W8_CASE
    return hipErrorInvalidValue;
}

}  // namespace vdb
