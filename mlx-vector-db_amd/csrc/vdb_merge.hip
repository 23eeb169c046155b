// vdb_merge.hip: merging sorted per-workgroup / per-shard top-k lists and the
// final result write-out (part of the gfx950 search pipeline, see vdb_scan.hip).
// Built with -ffp-contract=off.
#include "vdb_common.h"
#include "vdb_internal.h"
#include "vdb_merge_block.h"

namespace vdb {

// One workgroup (256 threads) per query (vdb_merge_block.h).
template <typename K, typename I>
__global__ void __launch_bounds__(256)
merge_lists_kernel(const K* __restrict__ ls, const I* __restrict__ li, int n_lists, int Lk, int64_t sq, int64_t sj,
                   int KP, K* __restrict__ out_k, I* __restrict__ out_i, const int* __restrict__ qcount) {
    if (qcount && (int)blockIdx.x >= *qcount) return;  // device-gated launch: only the flagged queries
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int q = blockIdx.x;
    merge_block<K, I>(ls + q * sq, li + q * sq, n_lists, Lk, sj, KP, out_k + (size_t)q * KP, out_i + (size_t)q * KP,
                      smem);
}

template <typename K, typename I>
static hipError_t merge_launch(int KP, const K* lk, const I* li, int n_lists, int Lk, int64_t sq, int64_t sj, int nq,
                               K* ok, I* oi, hipStream_t st, const int* qcount = nullptr) {
    if (KP < 32 || KP > 4096 || (KP & (KP - 1))) return hipErrorInvalidValue;
    const size_t lds = merge_block_lds<K, I>(KP);
    hipLaunchKernelGGL((merge_lists_kernel<K, I>), dim3(nq), dim3(256), lds, st, lk, li, n_lists, Lk, sq, sj, KP, ok,
                       oi, qcount);
    return hipGetLastError();
}

hipError_t launch_merge_f32(int KP, const float* ls, const uint32_t* li, int n_lists, int B, float* out_s,
                            uint32_t* out_i, hipStream_t st) {
    return merge_launch<float, uint32_t>(KP, ls, li, n_lists, KP, (int64_t)n_lists * KP, KP, B, out_s, out_i, st);
}

hipError_t launch_merge_f64_u32(int KP, const double* lk, const uint32_t* li, int n_lists, int Lk, int64_t sq,
                                int64_t sj, int nq, double* out_k, uint32_t* out_i, hipStream_t st, const int* qcount) {
    return merge_launch<double, uint32_t>(KP, lk, li, n_lists, Lk, sq, sj, nq, out_k, out_i, st, qcount);
}

hipError_t launch_merge_f64_i64(int KP, const double* lk, const int64_t* li, int n_lists, int Lk, int64_t sq,
                                int64_t sj, int nq, double* out_k, int64_t* out_i, hipStream_t st) {
    return merge_launch<double, int64_t>(KP, lk, li, n_lists, Lk, sq, sj, nq, out_k, out_i, st);
}

// Final results for query rows qmap[q] (or q) from sorted [nq][KP] lists.
template <typename I>
__global__ void __launch_bounds__(256) finalize_kernel(int metric, const double* __restrict__ sk,
                                                       const I* __restrict__ si, int KP, int nq,
                                                       const int* __restrict__ qmap, int k, int64_t index_offset,
                                                       float* __restrict__ out_s, int64_t* __restrict__ out_i,
                                                       double* __restrict__ out_k, const int* __restrict__ qcount,
                                                       const int64_t* __restrict__ row_ids) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= (int64_t)nq * k) return;
    const int qi = (int)(t / k);
    if (qcount && qi >= *qcount) return;  // device-gated launch
    const int e = (int)(t % k);
    const int b = qmap ? qmap[qi] : qi;
    const double key = sk[(size_t)qi * KP + e];
    const I ix = si[(size_t)qi * KP + e];
    const bool valid = sizeof(I) == 8 ? (int64_t)ix >= 0 : (uint32_t)ix != 0xFFFFFFFFu;
    const size_t o = (size_t)b * k + e;
    write_result(metric, key, valid ? global_row(row_ids, (uint64_t)ix, index_offset) : 0, valid && key != -INFINITY,
                 out_s + o, out_i + o, out_k ? out_k + o : nullptr);
}

// "No result" in every slot: what write_result stores for an invalid entry (score 0, row -1,
// key -inf), so a search of an empty index (or an empty shard of a row-sharded corpus) ranks
// below every real row in a later merge by key.
__global__ void __launch_bounds__(256) empty_results_kernel(int64_t n, float* __restrict__ out_s,
                                                            int64_t* __restrict__ out_i, double* __restrict__ out_k) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= n) return;
    write_result(0, 0.0, 0, false, out_s + t, out_i + t, out_k ? out_k + t : nullptr);
}

hipError_t launch_empty_results(int64_t n, float* out_s, int64_t* out_i, double* out_k, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(empty_results_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, n, out_s, out_i,
                       out_k);
    return hipGetLastError();
}

// Re-pass plumbing (vdb_api.cpp repass_flagged): the listed query rows gathered into a dense
// block, and the sub-search's result rows scattered back to those rows.
__global__ void __launch_bounds__(256) gather_rows_kernel(const float* __restrict__ Q, int D,
                                                          const int* __restrict__ list, int n, float* __restrict__ out) {
    const int r = blockIdx.y;
    const int b = list[r];
    for (int d = blockIdx.x * 256 + threadIdx.x; d < D; d += gridDim.x * 256) out[(size_t)r * D + d] = Q[(size_t)b * D + d];
}

hipError_t launch_gather_rows(const float* Q, int D, const int* list, int n, float* out, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)std::min(8, (D + 255) / 256), (unsigned)n), dim3(256), 0, st,
                       Q, D, list, n, out);
    return hipGetLastError();
}

__global__ void __launch_bounds__(256) repass_gather_kernel(const float* __restrict__ Q, int D,
                                                            const int* __restrict__ flags, int R,
                                                            float* __restrict__ out, int* __restrict__ counts,
                                                            unsigned long long* __restrict__ totals) {
    const int c = flags[0];
    const int n = c < R ? c : R;
    const int r = blockIdx.y;
    if (r == 0 && blockIdx.x == 0 && threadIdx.x == 0) {
        counts[0] = n;
        counts[1] = c > R ? c - R : 0;
        if (totals && n > 0) atomicAdd(totals, (unsigned long long)n);
    }
    // Slots past the gathered count are zeroed: the gated sub-search's query prep runs
    // over all R slots, and prep8 takes the batch's int8 scale as the maximum over every slot --
    // stale workspace bytes there (an earlier search's scores or ids) would coarsen it.
    if (r >= n) {
        for (int d = blockIdx.x * 256 + threadIdx.x; d < D; d += gridDim.x * 256) out[(size_t)r * D + d] = 0.0f;
        return;
    }
    const int b = flags[1 + r];
    for (int d = blockIdx.x * 256 + threadIdx.x; d < D; d += gridDim.x * 256) out[(size_t)r * D + d] = Q[(size_t)b * D + d];
}

hipError_t launch_repass_gather(const float* Q, int D, const int* flags, int R, float* out, int* counts,
                                unsigned long long* totals, hipStream_t st) {
    if (R <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(repass_gather_kernel, dim3((unsigned)std::min(8, (D + 255) / 256), (unsigned)R), dim3(256), 0,
                       st, Q, D, flags, R, out, counts, totals);
    return hipGetLastError();
}

__global__ void __launch_bounds__(256) scatter_results_kernel(const int* __restrict__ list, int n, int k,
                                                              const float* __restrict__ ss, const int64_t* __restrict__ si,
                                                              const double* __restrict__ sk, float* __restrict__ os,
                                                              int64_t* __restrict__ oi, double* __restrict__ ok,
                                                              const int* __restrict__ n_dev) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (n_dev && *n_dev < n) n = *n_dev;  // device re-pass: the gathered count
    if (t >= (int64_t)n * k) return;
    const int r = (int)(t / k), e = (int)(t % k);
    const size_t o = (size_t)list[r] * k + e;
    os[o] = ss[t];
    oi[o] = si[t];
    if (ok) ok[o] = sk[t];
}

hipError_t launch_scatter_results(const int* list, int n, int k, const float* ss, const int64_t* si, const double* sk,
                                  float* os, int64_t* oi, double* ok, hipStream_t st, const int* n_dev) {
    const int64_t m = (int64_t)n * k;
    if (m <= 0) return hipSuccess;
    hipLaunchKernelGGL(scatter_results_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, list, n, k, ss, si,
                       sk, os, oi, ok, n_dev);
    return hipGetLastError();
}

hipError_t launch_finalize_u32(int metric, const double* sk, const uint32_t* si, int KP, int nq, const int* qmap,
                               int k, int64_t index_offset, float* out_s, int64_t* out_i, double* out_k,
                               hipStream_t st, const int* qcount, const int64_t* row_ids) {
    const int64_t n = (int64_t)nq * k;
    hipLaunchKernelGGL(finalize_kernel<uint32_t>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, metric, sk, si,
                       KP, nq, qmap, k, index_offset, out_s, out_i, out_k, qcount, row_ids);
    return hipGetLastError();
}

hipError_t launch_finalize_i64(int metric, const double* sk, const int64_t* si, int KP, int nq, const int* qmap,
                               int k, float* out_s, int64_t* out_i, double* out_k, hipStream_t st) {
    const int64_t n = (int64_t)nq * k;
    hipLaunchKernelGGL(finalize_kernel<int64_t>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, metric, sk, si,
                       KP, nq, qmap, k, (int64_t)0, out_s, out_i, out_k, (const int*)nullptr, (const int64_t*)nullptr);
    return hipGetLastError();
}

}  // namespace vdb
