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
#include <algorithm>
#include "vdb_internal.h"

namespace vdb {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// ---- corpus / query tiling -------------------------------------------------
// A "row tile" is 32 rows, a "super tile" 4 row tiles (128 rows), a "group" 8
// dimensions.  Block (super tile st, group g, sub tile u) is 1 KiB in MFMA lane
// order: lane l holds the 4 floats
//   X[128 st + 32 u + (l & 31)][8 g + 4 (l >> 5) + j],  j = 0..3
// so one global_load_dwordx4 per lane fetches exactly the A operand of four
// consecutive v_mfma_f32_32x32x2_f32 k-steps (k index = l >> 5); a whole wave
// reads 1 KiB of contiguous HBM, and the 4 sub tiles of one group are adjacent
// (a wave owning several row tiles addresses them with immediate offsets).
// Layout: [T/4][G][4][64][4].  Dimensions are padded to Dp (multiple of 64,
// zeros), rows to the capacity (multiple of ROW_ALIGN, zeros).  Queries use the
// same layout.
__device__ __forceinline__ size_t tiled_block(uint64_t t, int g, int G) {
    return (((size_t)(t >> 2) * G + g) * 4 + (t & 3)) * BLOCK_FLOATS;
}

__device__ __forceinline__ size_t tiled_offset(uint64_t r, int d, int G) {
    const int i = (int)(r & 31);
    const int kk = (d >> 2) & 1;
    return tiled_block(r >> 5, d >> 3, G) + (i + 32 * kk) * 4 + (d & 3);
}

// Split-bf16 corpus / query tiles (PREC_BF16X3): a group is 16 dims; block
// (super tile st, group g, plane pl, sub tile u) is 1 KiB in the A/B operand
// order of v_mfma_f32_32x32x16_bf16: lane l holds the 8 bf16
//   plane(X[128 st + 32 u + (l & 31)][16 g + 8 (l >> 5) + j]),  j = 0..7
// plane 0 = hi = bf16(x), plane 1 = lo = bf16(x - hi).  Layout [T/4][G16][2][4][64][8];
// one (super tile, group) is 8 KiB contiguous.  Offsets in float units.
__device__ __forceinline__ size_t split_block(uint64_t t, int g, int G16) {
    return (((size_t)(t >> 2) * G16 + g) * 8 + (t & 3)) * BLOCK_FLOATS;
}
// The CORPUS copy's block of (tile t, group g, plane pl).  Default: the query layout above
// (the planes of a group adjacent).  VDB_PLANE_MAJOR: [T/4][2 planes][G16][4][1 KiB], so the hi
// plane of a super tile is G16 x 4 KiB contiguous (the bf16 pass reads only that plane).
#ifdef VDB_PLANE_MAJOR
constexpr bool kPlaneMajor = true;
#else
constexpr bool kPlaneMajor = false;
#endif
__host__ __device__ __forceinline__ size_t corpus_block(uint64_t t, int g, int pl, int G16) {
    if constexpr (kPlaneMajor) return ((((size_t)(t >> 2) * 2 + pl) * G16 + g) * 4 + (t & 3)) * BLOCK_FLOATS;
    return (((size_t)(t >> 2) * G16 + g) * 8 + 4 * pl + (t & 3)) * BLOCK_FLOATS;
}
// corpus offsets (floats) between consecutive groups / from the hi to the lo plane of a block
__host__ __device__ __forceinline__ constexpr size_t corpus_gstep() { return (kPlaneMajor ? 4 : 8) * BLOCK_FLOATS; }
__host__ __device__ __forceinline__ size_t corpus_plane(int G16) {
    return kPlaneMajor ? (size_t)G16 * 4 * BLOCK_FLOATS : 4 * BLOCK_FLOATS;
}

// Round-to-nearest-even fp32 -> bf16 bits for finite x (an overflow to inf falls
// back to truncation so that hi stays finite and hi + lo still tracks x).
__device__ __forceinline__ uint32_t bf16_rne_bits(float x) {
    const uint32_t u = __float_as_uint(x);
    const uint32_t r = (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
    return ((r & 0x7F80u) == 0x7F80u) ? (u >> 16) : r;
}

// x -> (hi, lo) bf16 pair, hi + lo = x within 2^-16 |x|
__device__ __forceinline__ void split_bf16(float x, uint32_t& hi, uint32_t& lo) {
    hi = bf16_rne_bits(x);
    lo = bf16_rne_bits(x - __uint_as_float(hi << 16));
}

// Pack 8 floats (two f32x4) into the hi / lo operand vectors (16 B each)
__device__ __forceinline__ void split8(const f32x4 a, const f32x4 b, f32x4& hi, f32x4& lo) {
    uint32_t h[8], l[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        split_bf16(a[j], h[j], l[j]);
        split_bf16(b[j], h[4 + j], l[4 + j]);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        hi[j] = __uint_as_float(h[2 * j] | (h[2 * j + 1] << 16));
        lo[j] = __uint_as_float(l[2 * j] | (l[2 * j + 1] << 16));
    }
}

// Order-preserving float <-> uint32 keys (0 = "no bound" = -inf): the shared
// per-query bounds are maintained with integer atomicMax.
__device__ __forceinline__ uint32_t order_key(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key_to_float(uint32_t k) {
    if (k == 0) return -INFINITY;
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

// LDS flags shared by a workgroup's waves (the flag-gated step ends of the candidate passes):
// relaxed workgroup-scope atomics keep the LDS address space (ds_read / ds_write).  A volatile
// access through a generic pointer compiled to flat_load / flat_store, which the compiler
// waits for with s_waitcnt vmcnt(0) -- at every step end, draining the corpus prefetch.
__device__ __forceinline__ int lds_flag_ld(int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_flag_st(int* p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
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
// oracle (oracle/ref_cpu.py, canonical_*) reproduces them bit for bit:
//   lane l owns the 4-dim "pieces" p = 64 m + l (dims 4p .. 4p+3), m = 0, 1, ...
//   (dims past D are zero; D is padded to a multiple of 256), and accumulates
//   them in (m, j) order with separate multiply and add (the library is built
//   with -ffp-contract=off); then an xor-butterfly over offsets 32,16,8,4,2,1.
// In the tiled corpus a piece is one aligned 16-byte load.
__device__ __forceinline__ double wave_sum_butterfly(double v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = v + __shfl_xor(v, off, 64);
    return v;
}

// float offset of piece p (dims 4p..4p+3) of row r in the tiled layout (fp32 candidate
// copy, query tiles)
__device__ __forceinline__ size_t tiled_piece_offset(uint64_t r, int p, int G) {
    return tiled_block(r >> 5, p >> 1, G) + (size_t)(r & 31) * 4 + (size_t)(p & 1) * 128;
}

// float offset of piece p of row r in the row-major fp32 corpus [cap][Dp] (Dp = 8 G): the
// exact paths gather whole rows, one coalesced 1 KiB load per wave per 256 dims
__device__ __forceinline__ size_t row_piece_offset(uint64_t r, int p, int G) {
    return (size_t)r * (size_t)(8 * G) + (size_t)p * 4;
}

// Global id of local row r: row_ids[r] (a shard of a multi-device set, whose rows are
// pieces of the global insertion order), else r + offset.
__device__ __forceinline__ uint64_t global_row(const int64_t* row_ids, uint64_t r, int64_t offset) {
    return row_ids ? (uint64_t)row_ids[r] : r + (uint64_t)offset;
}

// Write one result slot (fp32 score, int64 row, optional fp64 key).
__device__ __forceinline__ void write_result(int metric, double key, uint64_t row_plus_off, bool valid, float* os,
                                             int64_t* oi, double* ok) {
    if (valid) {
        *os = metric == 0 ? (float)key : (float)sqrt(-key);
        *oi = (int64_t)row_plus_off;
        if (ok) *ok = key;
    } else {
        *os = 0.0f;
        *oi = -1;
        if (ok) *ok = -INFINITY;
    }
}

// ---- LDS-resident sorting / streaming selection (runtime sizes, one wave) --------
// Used where a register network would be large (hundreds+ of elements): the
// loops are not unrolled, so code size and compile time stay small.  Only the
// calling wave touches the buffer; LDS accesses of one wave complete in order,
// the wave_barrier only stops the compiler from moving them across stages.
template <typename K, typename I>
__device__ __attribute__((noinline)) void wave_lds_sort_desc(K* k, I* ix, int n /* power of two */) {
    const int lane = threadIdx.x & 63;
    for (int size = 2; size <= n; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int e = lane; e < (n >> 1); e += 64) {
                const int lo = 2 * stride * (e / stride) + (e % stride);
                const int hi = lo + stride;
                const bool desc = (lo & size) == 0;
                const K a = k[lo], b = k[hi];
                const I ia = ix[lo], ib = ix[hi];
                const bool sw = desc ? better(b, ib, a, ia) : better(a, ia, b, ib);
                if (sw) {
                    k[lo] = b; k[hi] = a;
                    ix[lo] = ib; ix[hi] = ia;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }
    }
}

__host__ __device__ __forceinline__ int pow2_at_least(int v) {
    int p = 1;
    while (p < v) p <<= 1;
    return p;
}

// Streaming top-KP for ONE wave over batches of up to 64 candidates (one per
// lane), with an LDS buffer of capacity(KP) entries: candidates that beat the current
// threshold are appended; a full buffer is sorted and cut back to KP, which
// raises the threshold (the KP-th best so far).  Any KP (power of two).
template <typename K, typename I>
struct WaveTopK {
    K* bk;
    I* bi;
    int KP;
    int cap;  // buffer entries: power of two >= max(2 KP, KP + 64)
    int cnt;
    K tk;
    I ti;
    static __host__ __device__ int capacity(int kp) { return pow2_at_least(2 * kp > kp + 64 ? 2 * kp : kp + 64); }
    __device__ void init(K* k, I* i, int kp) {
        bk = k; bi = i; KP = kp; cap = capacity(kp); cnt = 0;
        tk = (K)-INFINITY; ti = sentinel_idx<I>();
    }
    __device__ void compact() {
        const int lane = threadIdx.x & 63;
        for (int e = cnt + lane; e < cap; e += 64) {
            bk[e] = (K)-INFINITY;
            bi[e] = sentinel_idx<I>();
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        wave_lds_sort_desc<K, I>(bk, bi, cap);
        cnt = cnt < KP ? cnt : KP;
        if (cnt == KP) {
            tk = bk[KP - 1];
            ti = bi[KP - 1];
        }
    }
    __device__ void offer(bool valid, K key, I idx) {
        const int lane = threadIdx.x & 63;
        bool pass = valid && better(key, idx, tk, ti);
        unsigned long long m = __ballot(pass);
        if (m == 0) return;
        if (cnt + __popcll(m) > cap) {
            compact();
            pass = valid && better(key, idx, tk, ti);
            m = __ballot(pass);
        }
        const int pos = cnt + __popcll(m & ((1ull << lane) - 1ull));
        if (pass) {
            bk[pos] = key;
            bi[pos] = idx;
        }
        cnt += __popcll(m);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    // sort what is kept; afterwards bk[0..min(cnt,KP)) is the sorted result and
    // the rest of [0, KP) holds sentinels
    __device__ void finish() { compact(); }
};

}  // namespace vdb
