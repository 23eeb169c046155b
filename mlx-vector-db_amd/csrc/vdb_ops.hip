// vdb_ops.hip — the reference's stand-alone similarity operators (the "operator slot"
// and performance/mlx_optimized.py), on gfx950:
//
//   sim_gemm_kernel   cosine / dot-product score matrix out[B][N] = Q X^T as an fp32 MFMA
//                     GEMM (v_mfma_f32_32x32x2_f32), corpus and query tiles staged through
//                     LDS from row-major memory, norms folded into the epilogue
//                     (compute_cosine_similarity_single/_batch, mlx_optimized.py:26-88;
//                     _compiled_cosine_similarity, service/optimized_vector_store.py:31-41;
//                     compute_dot_product, mlx_optimized.py:150-156);
//   l2_matrix_kernel  euclidean sqrt(sum((x - q)^2)) by direct differences, the reference's own
//                     form (mlx_optimized.py:139-148, optimized_vector_store.py:43-48): the
//                     expansion |x|^2 + |q|^2 - 2 q.x cancels for near rows;
//   normalize_kernel  x / max(|x|, 1e-8) (normalize_vectors, mlx_optimized.py:110-125);
//   topk kernels      top-k of arbitrary score rows, ties to the lower index
//                     (fast_top_k_indices / argsort(-s)[:k], mlx_optimized.py:90-108).
//
// These serve the reference's operator API; the store's search never materialises scores
// (vdb_scan.hip fuses scoring into the top-k).  Built with -ffp-contract=off.
#include "vdb_common.h"
#include "vdb_internal.h"

namespace vdb {

// ---- cosine / dot product score matrix (MFMA) ---------------------------------------------
// Workgroup: 4 waves, a 128-row x 32-query output tile (each wave 32 x 32); K loop over 32-dim
// slabs staged in LDS (rows padded to 33 floats: conflict-free column reads for the A / B
// operands of v_mfma_f32_32x32x2_f32: lane l reads row l & 31, dim k + (l >> 5)).
template <int METRIC>
__global__ void __launch_bounds__(256) sim_gemm_kernel(const float* __restrict__ X, int64_t N, int D,
                                                       const float* __restrict__ Q, int B, float* __restrict__ out) {
    __shared__ float sx[128][33];
    __shared__ float sq[32][33];
    __shared__ float so[4][32][33];
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int64_t r0 = (int64_t)blockIdx.x * 128;
    const int q0 = blockIdx.y * 32;
    f32x16 acc;
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[v] = 0.0f;
    float xs = 0.0f, qs = 0.0f;  // sum of squares of row (wv*32 + lane) / query lane (lanes < 32)
    for (int d0 = 0; d0 < D; d0 += 32) {
        for (int e = threadIdx.x; e < 128 * 32; e += 256) {
            const int r = e >> 5, c = e & 31;
            const int64_t row = r0 + r;
            sx[r][c] = (row < N && d0 + c < D) ? X[row * D + d0 + c] : 0.0f;
        }
        for (int e = threadIdx.x; e < 32 * 32; e += 256) {
            const int r = e >> 5, c = e & 31;
            sq[r][c] = (q0 + r < B && d0 + c < D) ? Q[(int64_t)(q0 + r) * D + d0 + c] : 0.0f;
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < 32; kk += 2) {
            const float a = sx[wv * 32 + (lane & 31)][kk + (lane >> 5)];
            const float b = sq[lane & 31][kk + (lane >> 5)];
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
        }
        if (METRIC == 0 && lane < 32) {
#pragma unroll 8
            for (int c = 0; c < 32; ++c) {
                const float xv = sx[wv * 32 + lane][c], qv = sq[lane][c];
                xs = fmaf(xv, xv, xs);
                qs = fmaf(qv, qv, qs);
            }
        }
        __syncthreads();
    }
    // accumulator lane l, register v: row (v & 3) + 8 (v >> 2) + 4 (l >> 5), query l & 31
    const float invx = 1.0f / fmaxf(sqrtf(xs), 1e-8f);
    const float invq = 1.0f / fmaxf(sqrtf(__shfl(qs, lane & 31, 64)), 1e-8f);
#pragma unroll
    for (int v = 0; v < 16; ++v) {
        const int i = (v & 3) + 8 * (v >> 2) + 4 * (lane >> 5);
        float val = acc[v];
        if (METRIC == 0) val = val * __shfl(invx, i, 64) * invq;
        so[wv][lane & 31][i] = val;
    }
    __syncthreads();
    // 32 consecutive rows per query: one 128-B store per (wave, query, half)
    for (int j = lane >> 5; j < 32; j += 2) {
        const int q = q0 + j;
        const int64_t row = r0 + wv * 32 + (lane & 31);
        if (q < B && row < N) out[(int64_t)q * N + row] = so[wv][j][lane & 31];
    }
}

// ---- euclidean score matrix (direct differences) ----------------------------------------
__global__ void __launch_bounds__(256) l2_matrix_kernel(const float* __restrict__ X, int64_t N, int D,
                                                        const float* __restrict__ Q, int B, float* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= N) return;
    const float* x = X + r * D;
    for (int b = 0; b < B; ++b) {
        const float* q = Q + (int64_t)b * D;
        float acc = 0.0f;
        for (int d = lane; d < D; d += 64) {
            const float df = x[d] - q[d];
            acc = fmaf(df, df, acc);
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, 64);
        if (lane == 0) out[(int64_t)b * N + r] = sqrtf(acc);
    }
}

hipError_t launch_similarity_matrix(const float* X, int64_t N, int D, const float* Q, int B, int metric, float* out,
                                    hipStream_t st) {
    if (N <= 0 || B <= 0) return hipSuccess;
    if (metric == 1) {
        hipLaunchKernelGGL(l2_matrix_kernel, dim3((unsigned)((N + 3) / 4)), dim3(256), 0, st, X, N, D, Q, B, out);
    } else {
        const dim3 grid((unsigned)((N + 127) / 128), (unsigned)((B + 31) / 32));
        if (metric == 0)
            hipLaunchKernelGGL(sim_gemm_kernel<0>, grid, dim3(256), 0, st, X, N, D, Q, B, out);
        else
            hipLaunchKernelGGL(sim_gemm_kernel<2>, grid, dim3(256), 0, st, X, N, D, Q, B, out);
    }
    return hipGetLastError();
}

// ---- row normalisation ----------------------------------------------------------------------
__global__ void __launch_bounds__(256) normalize_kernel(const float* __restrict__ in, int64_t n, int D,
                                                        float* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= n) return;
    const float* x = in + r * D;
    float s = 0.0f;
    for (int d = lane; d < D; d += 64) s = fmaf(x[d], x[d], s);
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
    const float nr = fmaxf(sqrtf(s), 1e-8f);
    for (int d = lane; d < D; d += 64) out[r * D + d] = x[d] / nr;
}

hipError_t launch_normalize_rows(const float* in, int64_t n, int D, float* out, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(normalize_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, in, n, D, out);
    return hipGetLastError();
}

// ---- top-k of score rows --------------------------------------------------------------------
// Pass 1: workgroup (chunk c, row b) keeps the best KP of its TOPK_CHUNK scores (each wave a
// quarter through WaveTopK, then wave 0 folds the other three), written sorted to
// lists[b][c][KP]; keys are the scores (largest) or their negation (smallest), NaN last.
// Pass 2: merge_lists over the chunks (vdb_merge.hip), then the index / value write-out.
constexpr int TOPK_CHUNK = 16384;

__device__ __forceinline__ float topk_key(float s, int largest) {
    if (s != s) return -INFINITY;  // NaN sorts after every number
    return largest ? s : -s;
}

__global__ void __launch_bounds__(256) topk_chunk_kernel(const float* __restrict__ S, int64_t n, int KP, int largest,
                                                         float* __restrict__ lk, uint32_t* __restrict__ li) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int cap = WaveTopK<float, uint32_t>::capacity(KP);
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    float* bk = reinterpret_cast<float*>(smem) + (size_t)wv * cap;
    uint32_t* bi = reinterpret_cast<uint32_t*>(smem + (size_t)4 * cap * sizeof(float)) + (size_t)wv * cap;
    const int b = blockIdx.y;
    const int64_t c0 = (int64_t)blockIdx.x * TOPK_CHUNK;
    const int64_t c1 = c0 + TOPK_CHUNK < n ? c0 + TOPK_CHUNK : n;
    const float* row = S + (int64_t)b * n;
    WaveTopK<float, uint32_t> tk;
    tk.init(bk, bi, KP);
    for (int64_t e0 = c0 + wv * 64; e0 < c1; e0 += 256) {
        const int64_t e = e0 + lane;
        const bool in = e < c1;
        tk.offer(in, in ? topk_key(row[e], largest) : -INFINITY, in ? (uint32_t)e : 0xFFFFFFFFu);
    }
    tk.finish();
    __syncthreads();
    if (wv != 0) return;
    for (int w = 1; w < 4; ++w) {
        const float* ok = reinterpret_cast<float*>(smem) + (size_t)w * cap;
        const uint32_t* oi = reinterpret_cast<uint32_t*>(smem + (size_t)4 * cap * sizeof(float)) + (size_t)w * cap;
        for (int e0 = 0; e0 < KP; e0 += 64) {
            const int e = e0 + lane;
            const bool in = e < KP && oi[e] != 0xFFFFFFFFu;
            tk.offer(in, in ? ok[e] : -INFINITY, in ? oi[e] : 0xFFFFFFFFu);
        }
    }
    tk.finish();
    const size_t base = ((size_t)b * gridDim.x + blockIdx.x) * KP;
    for (int e = lane; e < KP; e += 64) {
        lk[base + e] = tk.bk[e];
        li[base + e] = tk.bi[e];
    }
}

__global__ void __launch_bounds__(256) topk_write_kernel(const float* __restrict__ S, int64_t n,
                                                         const uint32_t* __restrict__ mi, int KP, int rows, int k,
                                                         int64_t* __restrict__ out_idx, float* __restrict__ out_val) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= (int64_t)rows * k) return;
    const int b = (int)(t / k), e = (int)(t % k);
    const uint32_t ix = mi[(size_t)b * KP + e];
    const bool valid = ix != 0xFFFFFFFFu;
    out_idx[t] = valid ? (int64_t)ix : -1;
    if (out_val) out_val[t] = valid ? S[(int64_t)b * n + ix] : 0.0f;
}

int topk_kp(int k) { return pow2_at_least(k < 32 ? 32 : k); }

size_t topk_workspace_bytes(int64_t n, int rows, int k) {
    const int KP = topk_kp(k);
    const int64_t chunks = (n + TOPK_CHUNK - 1) / TOPK_CHUNK;
    return ((size_t)rows * chunks * KP + (size_t)rows * KP) * 8 + 1024;
}

hipError_t launch_topk_scores(const float* S, int rows, int64_t n, int k, int largest, int64_t* out_idx, float* out_val,
                              void* ws, hipStream_t st) {
    const int KP = topk_kp(k);
    const int64_t chunks = (n + TOPK_CHUNK - 1) / TOPK_CHUNK;
    char* p = (char*)ws;
    float* lk = (float*)p;
    uint32_t* li = (uint32_t*)(p + (size_t)rows * chunks * KP * 4);
    float* mk = (float*)(p + (size_t)rows * chunks * KP * 8);
    uint32_t* mi = (uint32_t*)((char*)mk + (size_t)rows * KP * 4);
    const size_t lds = (size_t)4 * WaveTopK<float, uint32_t>::capacity(KP) * 8;
    hipLaunchKernelGGL(topk_chunk_kernel, dim3((unsigned)chunks, rows), dim3(256), lds, st, S, n, KP, largest, lk, li);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    e = launch_merge_f32(KP, lk, li, (int)chunks, rows, mk, mi, st);
    if (e != hipSuccess) return e;
    const int64_t tot = (int64_t)rows * k;
    hipLaunchKernelGGL(topk_write_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, S, n, mi, KP, rows, k,
                       out_idx, out_val);
    return hipGetLastError();
}

}  // namespace vdb
