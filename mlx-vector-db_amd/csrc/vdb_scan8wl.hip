// vdb_scan8wl.hip — the wide int8 pass for LONG rows (round 6): the I8 cosine pass for rows of
// 16..48 groups of 32 dims (512..1536 dims) and batches of 129..256 queries (C3: 1M x 1536,
// B = 256).
//
// Why.  The 64-query shape (scan8_kernel) holds one query block in LDS (96 KiB at 1536 dims), so
// C3's 4 query blocks each stream the corpus: the row ranges are re-read through L2 four times
// (PMC: 2.14 GB per launch = 1.39x the 1.54 GB of the xh plane) and the scan runs at 0.41 of HBM
// (profiles/r06f_c3).  Here one workgroup of 8 waves holds ALL 256 queries, 32 per wave, each
// wave's query tiles in REGISTERS for the whole launch (48 groups x 4 = 192 VGPRs at 1536 dims),
// and the corpus is read from HBM once: each row tile (32 rows, G KiB) is staged into an LDS ring
// of NSLOT tiles by LDS-DMA (global_load_lds_dwordx4, vdb_scan8w.hip w8_glds), NSLOT - 1 tiles
// in flight ahead of the one being scored, and every wave streams the tile's G A-operand blocks
// from LDS into one accumulator chain (one v_mfma_i32_32x32x32_i8 per group).
//
// Candidates go straight into the (workgroup, query) segments of the global lists against the
// pilot's bound, exactly as the short-row wide pass (vdb_scan8w.hip: same segment layout W8_CH,
// same seg_cnt, same checksum words), so the finish reads them in its seg mode unchanged; tiles
// are dealt round-robin (tile t -> workgroup t mod n_seg).
#include "vdb_scan8_kernel.h"

namespace vdb {

template <bool NT>
__device__ __forceinline__ void w8l_glds(const void* gsrc, uint32_t lds) {
    uint32_t keep;
    if constexpr (NT)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(gsrc), "s"(lds) : "memory");
    else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(gsrc), "s"(lds) : "memory");
}

// an LDS read the compiler does not track (waited for by s_waitcnt lgkmcnt tied to its register)
__device__ __forceinline__ void w8l_ds_read(f32x4& x, uint32_t addr) {
    asm volatile("ds_read_b128 %0, %1" : "=v"(x) : "v"(addr));
}

constexpr int W8L_NW = 8;                  // waves per workgroup (two per SIMD)
constexpr int W8L_QB = W8L_NW * 32;        // queries per workgroup: 256
#ifndef VDB_W8L_PD
#define VDB_W8L_PD 4
#endif
constexpr int W8L_PD = VDB_W8L_PD;  // LDS reads in flight ahead of the MFMA chain
#ifndef VDB_W8L_SMAX
#define VDB_W8L_SMAX 4
#endif
constexpr int W8L_SMAX = VDB_W8L_SMAX;  // ring slots at most (8 for 768-dim rows: C2 429 K vs 440 K QPS at 4)

// Waves and tiles.  A batch of QT_N = ceil(B / 32) query tiles, one per wave, leaves 8 - QT_N waves
// idle (they only stage the corpus); with RL > 1 each query tile gets RL waves that score the ring's
// tiles in turn: a round of RL tiles per barrier, tile R RL + r to the query tile's r-th wave.
// A small batch then spreads its MFMA chains and insertions over RL waves (C2 rows, B = 64: RL = 2).
// Ring: as many whole rounds of row tiles as fit the LDS beside the counters, at most W8L_SMAX
// tiles (1536 dims: 3 tiles of 48 KiB; 768: 4 of 24 KiB), the rounds after the current one in flight.
// (RL > 1 also keeps its shared per-query counters in LDS: 2 KiB)
template <int RL>
__host__ __device__ constexpr int w8l_cnt_bytes() { return RL > 1 ? 2 * W8L_QB * 4 : 0; }
template <int G, int RL>
__host__ __device__ constexpr int w8l_nslot() {
    return ((160 * 1024 - w8l_cnt_bytes<RL>()) / (G * 1024) < W8L_SMAX ? (160 * 1024 - w8l_cnt_bytes<RL>()) / (G * 1024)
                                                                        : W8L_SMAX) / RL * RL;
}
template <int G, int RL>
__host__ __device__ constexpr size_t w8l_lds_bytes() { return (size_t)w8l_nslot<G, RL>() * G * 1024 + w8l_cnt_bytes<RL>(); }
// the round wait: this wave's loads of the Y rounds issued after the one about to be scored may
// stay in flight, then the workgroup barrier
template <int N>
__device__ __forceinline__ void w8l_wait_bar() { asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory"); }

template <int G, int RL, bool NT>
__global__ void __launch_bounds__(64 * W8L_NW, 1)
scan8wl_kernel(const float* __restrict__ Xq, const uint32_t* __restrict__ mask, const float* __restrict__ Qq,
               const float* __restrict__ lsl, const float* __restrict__ qscal, int64_t N, int B,
               float* __restrict__ gl_s, uint32_t* __restrict__ gl_i, int64_t gl_cap, uint32_t* __restrict__ seg_cnt,
               const uint32_t* __restrict__ gthr, uint32_t* __restrict__ chkp) {
    constexpr int NW = W8L_NW, NSLOT = w8l_nslot<G, RL>(), P = NSLOT / RL - 1;
    constexpr size_t TILE_B = (size_t)G * 1024;
    constexpr size_t GSTEP = 8 * BLOCK_FLOATS;
    constexpr int LPW = RL * G / NW;  // corpus blocks per wave and round
    static_assert((RL * G) % NW == 0, "a round's blocks spread evenly over the waves");
    static_assert(P >= 1 && (P - 1) * LPW <= 63, "ring / vmcnt range");
    extern __shared__ __attribute__((aligned(16))) char s_dyn[];
    int* s_seg = (int*)(s_dyn + NSLOT * TILE_B);  // [256] this workgroup's entries per query
    uint32_t* s_ck = (uint32_t*)(s_seg + W8L_QB);  // [256] its checksum words

    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int w = blockIdx.x, n_seg = gridDim.x;
    const int qtn = (B + 31) >> 5;
    const int qtile = wv % qtn, rl = wv / qtn;
    const int q0 = qtile * 32;             // this wave's queries q0 .. q0 + 31
    const bool active = rl < RL;           // (wave-uniform: the others only stage the corpus)
    const int64_t T = (N + 31) >> 5;
    const int my_tiles = T > w ? (int)((T - 1 - w) / n_seg + 1) : 0;
    const int n_rounds = (my_tiles + RL - 1) / RL;
    const uint32_t ring = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)s_dyn;

    if constexpr (RL > 1) {
        for (int i = threadIdx.x; i < W8L_QB; i += 64 * NW) {
            s_seg[i] = 0;
            s_ck[i] = 0u;
        }
    }
    // RL = 1: a query tile belongs to one wave, whose lanes l and l + 32 (the tile's two row
    // halves) count its entries together in a register; RL > 1: its waves share LDS counters
    int cnt = 0;

    // this wave's LPW blocks of round R: local tiles R RL .. R RL + RL - 1 into slots
    // (R mod NSLOT / RL) RL + i (one 32-bit remainder per round, not a 64-bit one per block)
    auto issue = [&](int R) {
        const int rs = (R % (NSLOT / RL)) * RL;
#pragma unroll
        for (int u = 0; u < LPW; ++u) {
            const int j = wv * LPW + u;
            const int i = j / G, g = j % G;
            const int m = R * RL + i;
            if (RL == 1 || m < my_tiles)
                w8l_glds<NT>(Xq + corpus_block((uint64_t)m * n_seg + w, g, 0, G) + lane * 4,
                             ring + (uint32_t)((rs + i) * TILE_B) + (uint32_t)(g * 1024));
        }
    };

    const float uH = qscal[0], invU = qscal[2];
    f32x4 qr[G];
    const int q = q0 + (lane & 31);
    const bool qok = active && q < B;
    const float thf = qok ? key_to_float(gthr[q]) : INFINITY;
    const int thc = qok ? h_floor(thf, lsl[q], invU) : INT_MAX;
    uint32_t ckh = 0u;
    if (active) {
        const float* qs = Qq + s2_blk((uint64_t)qtile, 0, G + QG_EXTRA) + lane * 4;
#pragma unroll
        for (int g = 0; g < G; ++g) qr[g] = *(const f32x4*)(qs + g * GSTEP);
    }
#pragma unroll
    for (int p = 0; p < P; ++p)
        if (p < n_rounds) issue(p);

    for (int R = 0; R < n_rounds; ++R) {
        // round R's blocks have landed: this wave's loads of the P - 1 rounds issued after it
        // (R + 1 .. R + P - 1; R + P is issued below) may stay in flight when they are whole
        // rounds (LPW each; near the end wait for all); after the barrier every wave's have, and
        // every wave is done with round R - 1, whose slots round R + P now refills
        if (P > 1 && R + P - 1 < n_rounds && (R + P) * RL <= my_tiles)
            w8l_wait_bar<(P - 1) * LPW>();
        else
            w8l_wait_bar<0>();
        if (R + P < n_rounds) issue(R + P);
        const int m = R * RL + rl;
        if (!active || m >= my_tiles) continue;
        const int64_t t = (int64_t)m * n_seg + w;
        i32x16 aH;
#pragma unroll
        for (int v = 0; v < 16; ++v) aH[v] = 0;
        // The A operands stream from LDS W8L_PD groups ahead of their MFMA through a rolling
        // window of W8L_PD + 1 registers.  The reads are inline asm with explicit waits tied to the
        // register each MFMA consumes: compiler-visible reads were rescheduled by hipcc's
        // register-pressure heuristic down to two in flight (each MFMA pair waited on its reads).
        constexpr int PD = W8L_PD, NB = PD + 1;
        const uint32_t sa = ring + (uint32_t)(((R % (NSLOT / RL)) * RL + rl) * TILE_B) + (uint32_t)lane * 16u;
        f32x4 xb[NB];
#pragma unroll
        for (int p = 0; p < PD; ++p) w8l_ds_read(xb[p], sa + (uint32_t)(p * 1024));
#pragma unroll
        for (int g = 0; g < G; ++g) {
            if (g < G - PD)
                asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(xb[g % NB]) : "n"(PD - 1));
            else if (g == G - PD)
                asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(xb[g % NB]));
            if (g < G - PD) w8l_ds_read(xb[(g + PD) % NB], sa + (uint32_t)((g + PD) * 1024));
            aH = __builtin_amdgcn_mfma_i32_32x32x32_i8(__builtin_bit_cast(i32x4, xb[g % NB]),
                                                       __builtin_bit_cast(i32x4, qr[g]), aH, 0, 0, 0);
        }
        // ---- epilogue: the tile test, the checksum, the rare insertions ----
        const bool hit = __builtin_amdgcn_ballot_w64(imax16(aH) > thc) != 0ull;
        if (chkp) {
            if ((t + 1) * 32 <= N) {
                ckh += hsum16(aH);
            } else {
#pragma unroll
                for (int v = 0; v < 16; ++v) {
                    const int64_t row = t * 32 + 8 * (v >> 2) + 4 * (lane >> 5) + (v & 3);
                    if (row < N) ckh += (uint32_t)aH[v];
                }
            }
        }
        if (hit) {
            const uint32_t cand = qok ? tile_valid16(mask, t, N, lane) : 0u;
            float sv[16];
            uint32_t pm = 0;
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                sv[v] = (float)aH[v] * uH;
                pm |= (sv[v] > thf ? 1u : 0u) << v;
            }
            pm &= cand;
            int pos = 0;
            if constexpr (RL == 1) {
                const int np = __builtin_popcount(pm);
                const int np_hi = __shfl_xor(np, 32, 64);  // (the other row half's)
                pos = cnt + (lane >= 32 ? np_hi : 0);
                cnt += np + np_hi;
            } else {
                if (pm != 0u) pos = atomicAdd(&s_seg[q], __builtin_popcount(pm));
            }
            const uint32_t rb = (uint32_t)(t * 32) + 4u * (uint32_t)(lane >> 5);
            float* ls = gl_s + (size_t)q * gl_cap + (size_t)w * W8_CH;
            uint32_t* li = gl_i + (size_t)q * gl_cap + (size_t)w * W8_CH;
            while (pm != 0u) {
                const int v = __builtin_ctz(pm);
                pm &= pm - 1u;
                float a_ = sv[0];
#pragma unroll
                for (int u = 1; u < 16; ++u) a_ = v == u ? sv[u] : a_;
                if (pos < W8_CH) {
                    ls[pos] = a_;
                    li[pos] = rb + (uint32_t)((v & 3) + 8 * (v >> 2));
                }
                ++pos;
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // the checksum's partial sums (the tile's two row halves, lanes l and l + 32; the RL waves of a
    // query tile) and this workgroup's entries per query (the finish's segment counts; > W8_CH =
    // overflowed): one word per (query, workgroup)
    if constexpr (RL == 1) {
        if (!active) return;
        if (lane < 32 && q < B) seg_cnt[(size_t)q * n_seg + w] = (uint32_t)cnt;
        if (chkp) {
            const uint32_t hsum = ckh + (uint32_t)__shfl_xor((int)ckh, 32, 64);
            if (lane < 32 && q < B) chkp[(size_t)q * n_seg + w] = hsum;
        }
        return;
    }
    if (active && chkp) {
        const uint32_t hsum = ckh + (uint32_t)__shfl_xor((int)ckh, 32, 64);
        if (lane < 32) atomicAdd(&s_ck[q], hsum);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < B; i += 64 * NW) {
        seg_cnt[(size_t)i * n_seg + w] = (uint32_t)s_seg[i];
        if (chkp) chkp[(size_t)i * n_seg + w] = s_ck[i];
    }
}

// ---- one wave per query tile (RL = 1: batches of > 128, rows of 1536 dims): a tile per barrier.
// (The round-based kernel above with RL = 1 ran C3 2-8% slower than this form, same box,
// profiles/r06_rl4; this is the round-6 kernel that took C3 to 494 K.)
constexpr int W8L1_SMAX = 6;

// ring slots: as many row tiles as fit the LDS beside the segment counters, at most W8L1_SMAX
// (1536 dims: 3 tiles of 48 KiB; 768: 6 of 24 KiB)
template <int G>
__host__ __device__ constexpr int w8l1_nslot() {
    return (160 * 1024 - W8L_QB * 4) / (G * 1024) < W8L1_SMAX ? (160 * 1024 - W8L_QB * 4) / (G * 1024) : W8L1_SMAX;
}
// the stage wait: this wave's loads of the Y tiles younger than the one about to be scored may stay
// in flight (LPW each), then the workgroup barrier
template <int N>
__device__ __forceinline__ void w8l1_wait_bar() { asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory"); }
template <int G>
__host__ __device__ constexpr size_t w8l1_lds_bytes() { return (size_t)w8l1_nslot<G>() * G * 1024 + (size_t)W8L_QB * 4; }

template <int G, bool NT>
__global__ void __launch_bounds__(64 * W8L_NW, 1)
scan8wl1_kernel(const float* __restrict__ Xq, const uint32_t* __restrict__ mask, const float* __restrict__ Qq,
               const float* __restrict__ lsl, const float* __restrict__ qscal, int64_t N, int B, float* __restrict__ gl_s, uint32_t* __restrict__ gl_i,
               int64_t gl_cap, uint32_t* __restrict__ seg_cnt, const uint32_t* __restrict__ gthr,
               uint32_t* __restrict__ chkp) {
    constexpr int NW = W8L_NW, NSLOT = w8l1_nslot<G>();
    constexpr size_t TILE_B = (size_t)G * 1024;
    constexpr size_t GSTEP = 8 * BLOCK_FLOATS;
    constexpr int LPW = G / NW;  // corpus blocks per wave and tile
    static_assert(G % NW == 0, "a tile's blocks spread evenly over the waves");
    extern __shared__ __attribute__((aligned(16))) char s_dyn[];
    int* s_seg = (int*)(s_dyn + NSLOT * TILE_B);  // [NW][32]: this workgroup's entries per query

    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int w = blockIdx.x, n_seg = gridDim.x;
    const int q0 = wv * 32;       // this wave's queries q0 .. q0 + 31
    const bool active = q0 < B;   // (wave-uniform: a wave past the batch only loads)
    const int64_t T = (N + 31) >> 5;
    const int64_t my_tiles = T > w ? (T - 1 - w) / n_seg + 1 : 0;
    const uint32_t ring = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)s_dyn;

    if (lane < 32) s_seg[wv * 32 + lane] = 0;

    // this wave's LPW blocks of local tile m into slot m mod NSLOT
    auto issue = [&](int64_t m) {
        const uint32_t sbase = ring + (uint32_t)((m % NSLOT) * TILE_B);
        const int64_t t = m * n_seg + w;
#pragma unroll
        for (int u = 0; u < LPW; ++u) {
            const int g = wv * LPW + u;
            w8l_glds<NT>(Xq + corpus_block((uint64_t)t, g, 0, G) + lane * 4, sbase + (uint32_t)(g * 1024));
        }
    };

    const float uH = qscal[0], invU = qscal[2];
    f32x4 qr[G];
    const int q = q0 + (lane & 31);
    const bool qok = active && q < B;
    const float thf = qok ? key_to_float(gthr[q]) : INFINITY;
    const int thc = qok ? h_floor(thf, lsl[q], invU) : INT_MAX;
    uint32_t ckh = 0u;
    if (active) {
        const float* qs = Qq + s2_blk((uint64_t)(q0 / 32), 0, G + QG_EXTRA) + lane * 4;
#pragma unroll
        for (int g = 0; g < G; ++g) qr[g] = *(const f32x4*)(qs + g * GSTEP);
    }
#pragma unroll
    for (int p = 0; p < NSLOT - 1; ++p)
        if (p < my_tiles) issue(p);

    for (int64_t m = 0; m < my_tiles; ++m) {
        // tile m's blocks have landed: this wave's younger loads (tiles m + 1 .. m + NSLOT - 2)
        // may stay in flight (LPW each; fewer issued near the end: wait for all then); after the
        // barrier every wave's have, and every wave is done with tile m - 1, whose slot tile
        // m + NSLOT - 1 now refills
        static_assert(NSLOT >= 2 && NSLOT <= 6 && (NSLOT - 2) * LPW <= 63, "vmcnt range");
        switch ((int)min<int64_t>(NSLOT - 2, my_tiles - 1 - m)) {
            case 4: w8l1_wait_bar<4 * LPW>(); break;
            case 3: w8l1_wait_bar<3 * LPW>(); break;
            case 2: w8l1_wait_bar<2 * LPW>(); break;
            case 1: w8l1_wait_bar<LPW>(); break;
            default: w8l1_wait_bar<0>(); break;
        }
        if (m + NSLOT - 1 < my_tiles) issue(m + NSLOT - 1);
        if (!active) continue;
        const int64_t t = m * n_seg + w;
        i32x16 aH;
#pragma unroll
        for (int v = 0; v < 16; ++v) aH[v] = 0;
        // The A operands stream from LDS W8L_PD groups ahead of their MFMA through a rolling
        // window of W8L_PD + 1 registers.  The reads are inline asm with explicit waits tied to the
        // register each MFMA consumes: compiler-visible reads were rescheduled by hipcc's
        // register-pressure heuristic down to two in flight (each MFMA pair waited on its reads).
        constexpr int PD = W8L_PD, NB = PD + 1;
        const uint32_t sa = ring + (uint32_t)((m % NSLOT) * TILE_B) + (uint32_t)lane * 16u;
        f32x4 xb[NB];
#pragma unroll
        for (int p = 0; p < PD; ++p) w8l_ds_read(xb[p], sa + (uint32_t)(p * 1024));
#pragma unroll
        for (int g = 0; g < G; ++g) {
            if (g < G - PD)
                asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(xb[g % NB]) : "n"(PD - 1));
            else if (g == G - PD)
                asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(xb[g % NB]));
            if (g < G - PD) w8l_ds_read(xb[(g + PD) % NB], sa + (uint32_t)((g + PD) * 1024));
            aH = __builtin_amdgcn_mfma_i32_32x32x32_i8(__builtin_bit_cast(i32x4, xb[g % NB]),
                                                       __builtin_bit_cast(i32x4, qr[g]), aH, 0, 0, 0);
        }
        // ---- epilogue: the tile test, the checksum, the rare insertions ----
        const bool hit = __builtin_amdgcn_ballot_w64(imax16(aH) > thc) != 0ull;
        if (chkp) {
            if ((t + 1) * 32 <= N) {
                ckh += hsum16(aH);
            } else {
#pragma unroll
                for (int v = 0; v < 16; ++v) {
                    const int64_t row = t * 32 + 8 * (v >> 2) + 4 * (lane >> 5) + (v & 3);
                    if (row < N) ckh += (uint32_t)aH[v];
                }
            }
        }
        if (hit) {
            const int ql = lane & 31;
            const uint32_t cand = qok ? tile_valid16(mask, t, N, lane) : 0u;
            float sv[16];
            uint32_t pm = 0;
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                sv[v] = (float)aH[v] * uH;
                pm |= (sv[v] > thf ? 1u : 0u) << v;
            }
            pm &= cand;
            int pos = 0;
            if (pm != 0u) pos = atomicAdd(&s_seg[wv * 32 + ql], __builtin_popcount(pm));
            const uint32_t rb = (uint32_t)(t * 32) + 4u * (uint32_t)(lane >> 5);
            float* ls = gl_s + (size_t)q * gl_cap + (size_t)w * W8_CH;
            uint32_t* li = gl_i + (size_t)q * gl_cap + (size_t)w * W8_CH;
            while (pm != 0u) {
                const int v = __builtin_ctz(pm);
                pm &= pm - 1u;
                float a_ = sv[0];
#pragma unroll
                for (int u = 1; u < 16; ++u) a_ = v == u ? sv[u] : a_;
                if (pos < W8_CH) {
                    ls[pos] = a_;
                    li[pos] = rb + (uint32_t)((v & 3) + 8 * (v >> 2));
                }
                ++pos;
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!active) return;
    // this workgroup's entries per query (the finish's segment counts; > W8_CH = overflowed: each
    // wave reads back only its own counters) and the checksum's partial sum: the tile's two row
    // halves (lanes l, l + 32), one word per (query, workgroup)
    if (lane < 32 && q < B) seg_cnt[(size_t)q * n_seg + w] = (uint32_t)s_seg[wv * 32 + lane];
    if (chkp) {
        const uint32_t hsum = ckh + (uint32_t)__shfl_xor((int)ckh, 32, 64);
        if (lane < 32 && q < B) chkp[(size_t)q * n_seg + w] = hsum;
    }
}

bool scan8wl_ok(int prec, int metric, int G8, int B) {
    return prec == PREC_I8 && metric == 0 && B >= 1 && B <= W8L_QB && (G8 == 16 || G8 == 24 || G8 == 32 || G8 == 48);
}

template <int G, int RL, bool NT>
static hipError_t scan8wl_launch(const float* Xq, const uint32_t* mask, const float* Qq, const float* lsl,
                                 const float* qscal, int64_t N, int B, int n_seg, float* gl_s, uint32_t* gl_i,
                                 int64_t gl_cap, uint32_t* seg_cnt, const uint32_t* gthr, uint32_t* chkp,
                                 hipStream_t st) {
    auto k = RL == 1 ? scan8wl1_kernel<G, NT> : scan8wl_kernel<G, RL, NT>;
    constexpr size_t lds = RL == 1 ? w8l1_lds_bytes<G>() : w8l_lds_bytes<G, RL>();
    static_assert(lds <= 160 * 1024, "LDS");
    static std::atomic<bool> lds_set{false};
    if (!lds_set.load()) {
        const hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        lds_set = true;
    }
    hipLaunchKernelGGL(k, dim3((unsigned)n_seg), dim3(64 * W8L_NW), lds, st, Xq, mask, Qq, lsl, qscal, N, B, gl_s, gl_i,
                       gl_cap, seg_cnt, gthr, chkp);
    return hipGetLastError();
}

// waves per query tile: 2 while the batch's query tiles leave half the waves idle and the ring
// holds two rounds of two tiles ahead (rows of <= 1024 dims), else 1
int scan8wl_rl(int G8, int B) {
#ifdef VDB_W8L_RL1
    return 1;
#else
    return (B + 31) / 32 <= W8L_NW / 2 && G8 <= 32 ? 2 : 1;
#endif
}

hipError_t launch_scan8wl(int prec, int metric, const float* Xq, const uint32_t* mask, const float* Qq,
                          const float* lsl, const float* qscal, int G8, int64_t N, int B, int n_seg, float* gl_s,
                          uint32_t* gl_i, int64_t gl_cap, uint32_t* seg_cnt, const uint32_t* gthr, uint32_t* chkp,
                          hipStream_t st) {
    if (!scan8wl_ok(prec, metric, G8, B) || n_seg <= 0 || gl_cap != (int64_t)n_seg * W8_CH) return hipErrorInvalidValue;
    const int rl = scan8wl_rl(G8, B);
    // one query block: the corpus is read once, non-temporal
#define W8L_CASE(GV, RLV)                                                                                          \
    if (G8 == GV && rl == RLV)                                                                                     \
        return scan8wl_launch<GV, RLV, true>(Xq, mask, Qq, lsl, qscal, N, B, n_seg, gl_s, gl_i, gl_cap, seg_cnt, gthr, \
                                             chkp, st);
    W8L_CASE(16, 1) W8L_CASE(24, 1) W8L_CASE(32, 1) W8L_CASE(48, 1)
    W8L_CASE(16, 2) W8L_CASE(24, 2) W8L_CASE(32, 2)
#undef W8L_CASE
    return hipErrorInvalidValue;
}

}  // namespace vdb
