// vdb_exact.hip: exact fp64 keys: candidate rerank + certificate, exact full scan — part of the gfx950 kernels of the brute-force distance + top-k path
// (pipeline overview: vdb_scan.hip).  Built with -ffp-contract=off.
#include "vdb_common.h"
#include "vdb_internal.h"

namespace vdb {

// =============================================================================
// Exact fp64 keys
// =============================================================================
// key(q, r): cosine  dot / (max(|q|,1e-8) * max(|x|,1e-8))
//            L2      -(sum (x-q)^2)
// in the canonical order (vdb_common.h).  One wave per (query, row); up to four
// 16-byte corpus pieces per lane in flight.
template <int METRIC>
__device__ __forceinline__ double exact_key(const float* __restrict__ q, double qn, const float* __restrict__ X, int G,
                                            int D, uint64_t r, double xn) {
    const int lane = threadIdx.x & 63;
    const int Dp = G * GROUP_DIMS;
    const int np = (D + 255) / 256;
    double acc = 0.0;
    for (int m0 = 0; m0 < np; m0 += 4) {
        f32x4 xv[4];
        float qv[4][4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int p = (m0 + u) * 64 + lane;
            const bool in = (m0 + u) < np;
            xv[u] = (in && 4 * p < Dp) ? *(const f32x4*)(X + tiled_piece_offset(r, p, G)) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int j = 0; j < 4; ++j) qv[u][j] = (in && 4 * p + j < D) ? q[4 * p + j] : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if ((m0 + u) < np) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const double qd = (double)qv[u][j];
                    const double xd = (double)xv[u][j];
                    if (METRIC == 0) {
                        acc = acc + qd * xd;
                    } else {
                        const double df = xd - qd;
                        acc = acc + df * df;
                    }
                }
            }
        }
    }
    acc = wave_sum_butterfly(acc);
    if (METRIC == 0) return acc / (fmax(qn, 1e-8) * fmax(xn, 1e-8));
    return -acc;
}

// Rerank: exact keys of the KP candidates (16 waves, one candidate per wave at a
// time), best k out, and the certificate that the exact top-k lies inside the
// candidate set:
//   every non-candidate row r has approx a_r <= a_KP (scan invariant), and
//   |approx - exact| <= eps, so if a_KP + eps < a_k - eps no non-candidate can
//   reach the top k.  A failed certificate queues the query for exact_scan.
constexpr int RERANK_WAVES = 16;

template <int METRIC, int KP>
__global__ void __launch_bounds__(64 * RERANK_WAVES) rerank_kernel(RerankArgs a) {
    constexpr int E = KP >= 64 ? KP / 64 : 1;
    __shared__ double s_k[KP];
    __shared__ uint32_t s_i[KP];
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int b = blockIdx.x;
    const float* q = a.Q + (int64_t)b * a.D;
    const double qn = a.qn64[b];
    for (int c = wv; c < KP; c += RERANK_WAVES) {
        const uint32_t r = a.app_i[(size_t)b * KP + c];
        double key = -INFINITY;
        if (r != 0xFFFFFFFFu) key = exact_key<METRIC>(q, qn, a.X, a.G, a.D, r, a.nrm64[r]);
        if (lane == 0) {
            s_k[c] = key;
            s_i[c] = r;
        }
    }
    __syncthreads();
    if (wv != 0) return;
    double kv[E];
    uint32_t iv[E];
#pragma unroll
    for (int i = 0; i < E; ++i) {
        const int e = i * 64 + lane;
        kv[i] = e < KP ? s_k[e] : -INFINITY;
        iv[i] = e < KP ? s_i[e] : 0xFFFFFFFFu;
    }
    wave_sort_desc<double, uint32_t, E>(kv, iv);
#pragma unroll
    for (int i = 0; i < E; ++i) {
        const int e = i * 64 + lane;
        if (e < a.k) {
            const size_t o = (size_t)b * a.k + e;
            write_result(METRIC, kv[i], (uint64_t)iv[i] + a.index_offset, iv[i] != 0xFFFFFFFFu, a.out_s + o,
                         a.out_i + o, a.out_k ? a.out_k + o : nullptr);
        }
    }
    if (lane == 0) {
        bool ok = true;
        if (a.app_i[(size_t)b * KP + KP - 1] != 0xFFFFFFFFu) {  // >= KP eligible rows: need the bound
            const double ak = (double)a.app_s[(size_t)b * KP + a.k - 1];
            const double akp = (double)a.app_s[(size_t)b * KP + KP - 1];
            double eps;
            if (METRIC == 0) {
                eps = a.eps_rel;
            } else {
                eps = a.eps_rel * (2.0 * qn * a.xmax + a.xmax * a.xmax) + 2.4e-7 * fmax(fabs(ak), fabs(akp));
            }
            ok = akp + eps < ak - eps;
        }
        if (!ok) {
            const int pos = atomicAdd(a.flag_count, 1);
            a.flag_list[pos] = b;
        }
    }
}

hipError_t launch_rerank(int metric, int KP, const RerankArgs& a, int B, hipStream_t st) {
#define VDB_RR(M, KPV)                                                                       \
    if (metric == M && KP == KPV) {                                                          \
        hipLaunchKernelGGL((rerank_kernel<M, KPV>), dim3(B), dim3(64 * RERANK_WAVES), 0, st, a);           \
        return hipGetLastError();                                                            \
    }
    VDB_RR(0, 32) VDB_RR(0, 64) VDB_RR(0, 128) VDB_RR(0, 256)
    VDB_RR(1, 32) VDB_RR(1, 64) VDB_RR(1, 128) VDB_RR(1, 256)
#undef VDB_RR
    return hipErrorInvalidValue;
}

// Exact scan (certificate fallback, and the path for k > 200): every eligible
// row of a workgroup's range gets its exact key (one wave per row); each wave
// streams its rows through a WaveTopK (LDS buffer), then wave 0 folds the other
// three waves' lists into its own and writes the workgroup's sorted top-KE.
template <int METRIC>
__global__ void __launch_bounds__(256)
exact_scan_kernel(const float* __restrict__ Q, const double* __restrict__ qn64, const int* __restrict__ qlist,
                  const float* __restrict__ X, int G, int D, const double* __restrict__ nrm64,
                  const uint32_t* __restrict__ mask, int64_t N, int64_t rows_per_wg, int KE,
                  double* __restrict__ lk, uint32_t* __restrict__ li) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int cap = WaveTopK<double, uint32_t>::capacity(KE);
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    double* bk = reinterpret_cast<double*>(smem) + (size_t)wv * cap;
    uint32_t* bi = reinterpret_cast<uint32_t*>(smem + (size_t)4 * cap * sizeof(double)) + (size_t)wv * cap;
    const int qi = blockIdx.y;
    const int b = qlist ? qlist[qi] : qi;
    const float* q = Q + (int64_t)b * D;
    const double qn = qn64[b];
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_wg;
    const int64_t r1 = r0 + rows_per_wg < N ? r0 + rows_per_wg : N;
    WaveTopK<double, uint32_t> tk;
    tk.init(bk, bi, KE);
    for (int64_t r = r0 + wv; r < r1; r += 4) {
        if (mask && !((mask[r >> 5] >> (r & 31)) & 1u)) continue;
        const double key = exact_key<METRIC>(q, qn, X, G, D, (uint64_t)r, nrm64[r]);
        tk.offer(lane == 0, key, (uint32_t)r);
    }
    tk.finish();
    __syncthreads();
    if (wv != 0) return;
    for (int w = 1; w < 4; ++w) {
        const double* ok = reinterpret_cast<double*>(smem) + (size_t)w * cap;
        const uint32_t* oi = reinterpret_cast<uint32_t*>(smem + (size_t)4 * cap * sizeof(double)) + (size_t)w * cap;
        for (int e0 = 0; e0 < KE; e0 += 64) {
            const int e = e0 + lane;
            const bool in = e < KE && oi[e] != 0xFFFFFFFFu;
            tk.offer(in, in ? ok[e] : -INFINITY, in ? oi[e] : 0xFFFFFFFFu);
        }
    }
    tk.finish();
    const size_t base = ((size_t)qi * gridDim.x + blockIdx.x) * KE;
    for (int e = lane; e < KE; e += 64) {
        lk[base + e] = bk[e];
        li[base + e] = bi[e];
    }
}

hipError_t launch_exact_scan(int metric, int KE, const float* Q, const double* qn64, const int* qlist, int nq,
                             const float* X, int G, int D, const double* nrm64, const uint32_t* mask, int64_t N,
                             int n_wg, int64_t rows_per_wg, double* lk, uint32_t* li, hipStream_t st) {
    const size_t lds = (size_t)4 * WaveTopK<double, uint32_t>::capacity(KE) * (sizeof(double) + sizeof(uint32_t));
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    if (metric == 0)
        hipLaunchKernelGGL((exact_scan_kernel<0>), dim3(n_wg, nq), dim3(256), lds, st, Q, qn64, qlist, X, G, D, nrm64,
                           mask, N, rows_per_wg, KE, lk, li);
    else
        hipLaunchKernelGGL((exact_scan_kernel<1>), dim3(n_wg, nq), dim3(256), lds, st, Q, qn64, qlist, X, G, D, nrm64,
                           mask, N, rows_per_wg, KE, lk, li);
    return hipGetLastError();
}

}  // namespace vdb
