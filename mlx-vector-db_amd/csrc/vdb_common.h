// vdb_common.h — device-side building blocks shared by the vdb kernels.
//
// Everything here is written for gfx950 (CDNA4): 64-lane wavefronts, fp32-in
// MFMA (v_mfma_f32_32x32x2_f32), and the ordering contract of the reference
// (score desc, row index asc — SURVEY.md §8 S4).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include <type_traits>
#include "vdb_internal.h"

namespace vdb {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// ---- corpus / query tiling -------------------------------------------------
// A "row tile" is 32 rows; a "group" is 8 dimensions.  Tile (t, g) is one
// 1 KiB block laid out in MFMA lane order: lane l holds the 4 floats
//   X[32 t + (l & 31)][8 g + 4 (l >> 5) + j],  j = 0..3
// so one global_load_dwordx4 per lane fetches exactly the A operand of four
// consecutive v_mfma_f32_32x32x2_f32 k-steps (k index = l >> 5), and a whole
// wave reads 1 KiB of contiguous HBM.  Dimensions are padded to Dp (multiple
// of 32, zeros), rows to the capacity (multiple of 256, zeros).
__device__ __forceinline__ size_t tiled_offset(uint64_t r, int d, int G) {
    const uint64_t t = r >> 5;
    const int i = (int)(r & 31);
    const int g = d >> 3;
    const int kk = (d >> 2) & 1;
    const int j = d & 3;
    return (((size_t)t * G + g) * 64 + i + 32 * kk) * 4 + j;
}

// ---- ordering ----------------------------------------------------------------
// Keys are "higher is better"; ties go to the LOWER row index.  Index types are
// compared unsigned so that the sentinel (UINT32_MAX / int64 -1) sorts last.
template <typename K, typename I>
__device__ __forceinline__ bool better(K as, I ai, K bs, I bi) {
    typedef typename std::conditional<sizeof(I) == 8, unsigned long long, unsigned int>::type U;
    return as > bs || (as == bs && (U)ai < (U)bi);
}

template <typename I> __device__ __forceinline__ I sentinel_idx();
template <> __device__ __forceinline__ uint32_t sentinel_idx<uint32_t>() { return 0xFFFFFFFFu; }
template <> __device__ __forceinline__ int64_t sentinel_idx<int64_t>() { return (int64_t)-1; }

template <typename T> __device__ __forceinline__ T shfl_xor_t(T v, int m) { return __shfl_xor(v, m, 64); }
template <typename T> __device__ __forceinline__ T shfl_t(T v, int src) { return __shfl(v, src, 64); }

// One compare-exchange stage of a bitonic network over a wave-resident array of
// 64*E elements (element e = i*64 + lane lives in register i of lane e&63).
// SIZE selects the direction of each block ((e & SIZE) == 0 -> descending,
// i.e. better first); SIZE >= 64*E means "everything descending".  SIZE and
// STRIDE are template parameters so every register index is a compile-time
// constant (a runtime index would send the arrays to scratch).
template <typename K, typename I, int E, int SIZE, int STRIDE>
__device__ __forceinline__ void bitonic_stage(K (&s)[E], I (&ix)[E]) {
    const int lane = threadIdx.x & 63;
    if constexpr (STRIDE >= 64) {
        constexpr int RS = STRIDE / 64;
#pragma unroll
        for (int i = 0; i < E; ++i) {
            if ((i & RS) == 0) {
                const int p = i | RS;
                const int e = i * 64 + lane;
                const bool desc = (e & SIZE) == 0;
                const bool sw = desc ? better(s[p], ix[p], s[i], ix[i]) : better(s[i], ix[i], s[p], ix[p]);
                if (sw) {
                    K tk = s[i]; s[i] = s[p]; s[p] = tk;
                    I ti = ix[i]; ix[i] = ix[p]; ix[p] = ti;
                }
            }
        }
    } else {
        const bool lower = (lane & STRIDE) == 0;
#pragma unroll
        for (int i = 0; i < E; ++i) {
            const K os = shfl_xor_t(s[i], STRIDE);
            const I oi = shfl_xor_t(ix[i], STRIDE);
            const int e = i * 64 + lane;
            const bool desc = (e & SIZE) == 0;
            const bool sw = (lower == desc) ? better(os, oi, s[i], ix[i]) : better(s[i], ix[i], os, oi);
            if (sw) { s[i] = os; ix[i] = oi; }
        }
    }
}

template <typename K, typename I, int E, int SIZE, int STRIDE>
__device__ __forceinline__ void bitonic_passes(K (&s)[E], I (&ix)[E]) {
    if constexpr (STRIDE > 0) {
        bitonic_stage<K, I, E, SIZE, STRIDE>(s, ix);
        bitonic_passes<K, I, E, SIZE, STRIDE / 2>(s, ix);
    }
}

// Full bitonic sort, best first, of 64*E wave-resident elements.
template <typename K, typename I, int E, int SIZE = 2>
__device__ __forceinline__ void wave_sort_desc(K (&s)[E], I (&ix)[E]) {
    if constexpr (SIZE <= 64 * E) {
        bitonic_passes<K, I, E, SIZE, SIZE / 2>(s, ix);
        wave_sort_desc<K, I, E, SIZE * 2>(s, ix);
    }
}

// Bitonic merge (all descending) of a 64*E bitonic sequence: strides n/2..1.
template <typename K, typename I, int E>
__device__ __forceinline__ void wave_merge_desc(K (&s)[E], I (&ix)[E]) {
    bitonic_passes<K, I, E, (1 << 30), 32 * E>(s, ix);
}

// ---- canonical fp64 arithmetic ---------------------------------------------------
// The exact ranking keys are computed in ONE fixed order so that the numpy
// oracle (oracle/ref_cpu.py: canonical_dot64) reproduces them bit for bit:
// lane l accumulates dims d = l, l+64, l+128, ... (zero beyond the data) with
// separate multiply and add (the file is built with -ffp-contract=off), then a
// xor-butterfly over offsets 32,16,8,4,2,1.
__device__ __forceinline__ double wave_sum_butterfly(double v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = v + __shfl_xor(v, off, 64);
    return v;
}

}  // namespace vdb
