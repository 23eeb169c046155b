// vdb_scan2.hip — the split-bf16 candidate pass (PREC_BF16X3, the default, and PREC_BF16):
// pilot kernel, dispatch to the instantiation units (kernel: vdb_scan2_kernel.h).
#include "vdb_scan2_kernel.h"

namespace vdb {

// =============================================================================
// Pilot bound with the same arithmetic (vdb_scan.hip launch_pilot for the fp32 pass)
// =============================================================================
// The pilot only has to produce a number: rows the candidate pass drops below the bound are
// covered by the certificate whatever the bound is (vdb_api.cpp pilot_rank), so the pilot
// splits a tile's dimension groups over W waves (a 1/W of the dependent load chain of a
// one-wave tile) and sums the partial accumulators through LDS; a 4-wave block scores 4/W
// tiles (W = 4 for long rows, fewer for short ones: C4's 8 groups per tile take W = 2, half
// the blocks of one tile per block).
constexpr int PILOT_WAVES = 4;

__host__ __device__ inline int pilot2_w(int G) { return G >= 16 ? 4 : G >= 6 ? 2 : 1; }

template <int PREC, int METRIC, int QT>
__global__ void __launch_bounds__(64 * PILOT_WAVES)
pilot2_scores_kernel(const float* __restrict__ Xs, const float* __restrict__ rinit, const uint32_t* __restrict__ mask,
                     const float* __restrict__ Qs, int G, int64_t N, int B, int64_t n_tiles, int n_sample,
                     uint32_t* __restrict__ pslots) {
    constexpr int QB = 32 * QT;
    constexpr int XPL = Planes<PREC>::XPL;
    constexpr size_t GSTEP = 8 * BLOCK_FLOATS, PLANE = 4 * BLOCK_FLOATS;
    __shared__ float s_part[PILOT_WAVES][QT][16][64];
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int W = pilot2_w(G);  // waves per tile (block-uniform)
    const int part = wv % W;    // this wave's share of the tile's groups
    const int i = blockIdx.x * (PILOT_WAVES / W) + wv / W;  // sample index
    const int qb = blockIdx.y;
    const bool live = i < n_sample;
    const uint64_t t = live ? (uint64_t)((int64_t)i * n_tiles / n_sample) : 0;
    const float* xs = Xs + corpus_block(t, 0, 0, G) + lane * 4;
    const size_t XGSTEP = corpus_gstep(), XPLANE = corpus_plane(G);
    const float* qs = Qs + s2_blk((uint64_t)(qb * QT), 0, G + QG_EXTRA) + lane * 4;
    f32x16 acc[1][QT];
    const float r1 = (METRIC == 1 && part == 0 && lane < 32) ? rinit[t * 32 + lane] : 0.0f;
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[0][qt][v] = 0.0f;
        if (METRIC == 1) acc[0][qt] = __builtin_amdgcn_mfma_f32_32x32x2f32(r1, lane < 32 ? 1.0f : 0.0f, acc[0][qt], 0, 0, 0);
    }
    // groups part, part + W, ...; PP of them in flight
    constexpr int PP = 4;
    f32x4 xr[PP][1][XPL], qr[PP][QT][2];
    auto load = [&](int slot, int g) {
        if (g < G) {
#pragma unroll
            for (int pl = 0; pl < XPL; ++pl) xr[slot][0][pl] = *(const f32x4*)(xs + g * XGSTEP + pl * XPLANE);
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                for (int pl = 0; pl < 2; ++pl)
                    qr[slot][qt][pl] = *(const f32x4*)(qs + g * GSTEP + pl * PLANE + qt * BLOCK_FLOATS);
        }
    };
#pragma unroll
    for (int p = 0; p < PP; ++p) load(p, part + W * p);
    for (int g0 = part; g0 < G; g0 += W * PP) {
#pragma unroll
        for (int p = 0; p < PP; ++p) {
            const int g = g0 + W * p;
            if (g < G) {
                group_mfma<PREC, 1, QT>(xr[p], qr[p], acc);
                load(p, g + W * PP);
            }
        }
    }
    if (part > 0) {
#pragma unroll
        for (int qt = 0; qt < QT; ++qt)
#pragma unroll
            for (int v = 0; v < 16; ++v) s_part[wv][qt][v][lane] = acc[0][qt][v];
    }
    __syncthreads();
    if (part > 0 || !live) return;
    for (int w = 1; w < W; ++w)
#pragma unroll
        for (int qt = 0; qt < QT; ++qt)
#pragma unroll
            for (int v = 0; v < 16; ++v) acc[0][qt][v] += s_part[wv + w][qt][v][lane];
    const uint32_t valid = tile_valid16(mask, (int64_t)t, N, lane);
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
        const int q = qb * QB + qt * 32 + (lane & 31);
        float best = -INFINITY;
#pragma unroll
        for (int v = 0; v < 16; ++v) best = ((valid >> v) & 1u) ? fmaxf(best, acc[0][qt][v]) : best;
        if (METRIC == 1) best = 2.0f * best;
        best = fmaxf(best, __shfl_xor(best, 32, 64));  // the tile's two row halves (lane, lane + 32)
        if (lane < 32 && q < B && best != -INFINITY) atomicMax(pslots + pslot_at(q, i % PILOT_SLOTS, B), order_key(best));
    }
}

hipError_t launch_pilot2(int prec, int metric, int KP, const float* Xs, const float* rinit, const uint32_t* mask,
                         const float* Qs, int G, int64_t N, int B, int n_qblocks, int QB, int n_sample,
                         uint32_t* pslots, uint32_t* gthr, hipStream_t st) {
    const int64_t n_tiles = (N + 31) / 32;
    if (n_sample > n_tiles) n_sample = (int)n_tiles;
    if (n_sample <= 0 || KP > PILOT_SLOTS) return hipSuccess;
    const int tpb = PILOT_WAVES / pilot2_w(G);  // tiles per block
    const dim3 grid((n_sample + tpb - 1) / tpb, n_qblocks);
    bool launched = false;
#define VDB_PILOT2(P, M, QTV)                                                                                     \
    if (!launched && prec == P && metric == M && QB == 32 * QTV) {                                                \
        hipLaunchKernelGGL((pilot2_scores_kernel<P, M, QTV>), grid, dim3(64 * PILOT_WAVES), 0, st, Xs, rinit, mask, \
                           Qs, G, N, B, n_tiles, n_sample, pslots);                                               \
        launched = true;                                                                                          \
    }
    VDB_PILOT2(1, 0, 2) VDB_PILOT2(1, 1, 2) VDB_PILOT2(1, 0, 1) VDB_PILOT2(1, 1, 1)
    VDB_PILOT2(2, 0, 2) VDB_PILOT2(2, 1, 2) VDB_PILOT2(2, 0, 1) VDB_PILOT2(2, 1, 1)
#undef VDB_PILOT2
    if (!launched) return hipErrorInvalidValue;
    (void)KP;
    (void)gthr;  // the bound itself is taken by the candidate pass (scan2_kernel, pilot_slot_rank)
    return hipGetLastError();
}

// =============================================================================
// Dispatch
// =============================================================================
int scan2_rows_per_step(bool q4) { return q4 ? 2 * S2_NW * 32 : S2_ROWS; }

hipError_t launch_scan2(int prec, int metric, int KP, const float* Xs, const float* rinit, const uint32_t* mask,
                        const float* Qs, int G, int64_t N, int B, int n_qblocks, int64_t n_steps, int n_wg, int spw,
                        float* gl_s, uint32_t* gl_i, uint32_t* gl_cnt, int64_t gl_cap, uint32_t* gthr,
                        int lockstep, hipStream_t st, bool q4, int qlds, const int* gate) {
    // the query block in LDS: auto (qlds < 0) when it fits, 0 = from global memory (then, with one
    // query block, the corpus stream takes the non-temporal policy)
    const bool ql = q4 || (qlds != 0 && scan2_qlds(G, KP, q4));
    if (q4 && (!ql || KP != 128)) return hipErrorInvalidValue;
    const bool fs = !lockstep;
    const bool nt = !ql && n_qblocks == 1;
    auto* unit = prec == PREC_BF16X3 ? (metric == 0 ? launch_scan2_b3c : launch_scan2_b3l)
                 : prec == PREC_BF16 ? (metric == 0 ? launch_scan2_b1c : launch_scan2_b1l)
                                     : nullptr;
    if (!unit || metric < 0 || metric > 1) return hipErrorInvalidValue;
    return unit(KP, Xs, rinit, mask, Qs, G, N, B, n_qblocks, n_steps, n_wg, spw, gl_s, gl_i, gl_cnt, gl_cap, gthr, nt,
                ql, fs, q4, gate, st);
}

}  // namespace vdb
