// vdb_kernels.hip — gfx950 kernels of the brute-force distance + top-k path.
//
// Pipeline for one search:
//   prep_queries  -> scan_topk (fp32 MFMA candidate pass, fused per-WG top-KP)
//   -> merge_lists (per-query top-KP over all WG lists)
//   -> rerank (exact fp64 keys of the KP candidates, top-k, certificate)
//   -> [rare] exact_scan + merge + finalize for queries whose certificate failed.
//
// Reference semantics restated here (file:line in /root/reference):
//   cosine  = (q/max(|q|,1e-8)).(x/max(|x|,1e-8))   service/optimized_vector_store.py:31-41
//   L2      = sqrt(sum((x-q)^2))                    service/optimized_vector_store.py:43-48
//   order   = argsort(-score)[:k] / argsort(dist)[:k], ties -> lower row
//                                                   service/optimized_vector_store.py:176-183
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off (fp64 canonical order).
#include "vdb_common.h"
#include "vdb_internal.h"

namespace vdb {

// =============================================================================
// Ingest
// =============================================================================
// One wave per row.  Canonical fp64 norm (see vdb_common.h), tiled store.
__global__ void __launch_bounds__(256) pack_rows_kernel(const float* __restrict__ src, int64_t n, int D, int G,
                                                        float* __restrict__ X, int64_t row0,
                                                        double* __restrict__ nrm64, float* __restrict__ inv32,
                                                        float* __restrict__ sq32,
                                                        unsigned long long* __restrict__ xmax_bits,
                                                        int* __restrict__ nonfinite) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n) return;
    const int Dp64 = (D + 63) & ~63;
    const float* s = src + row * (int64_t)D;
    const uint64_t r = (uint64_t)(row0 + row);
    double acc = 0.0;
    int bad = 0;
    for (int d = lane; d < Dp64; d += 64) {
        const float v = d < D ? s[d] : 0.0f;
        bad |= !isfinite(v);
        const double dv = (double)v;
        acc = acc + dv * dv;
        if (d < D) X[tiled_offset(r, d, G)] = v;
    }
    acc = wave_sum_butterfly(acc);
    const int anybad = __any(bad);
    if (lane == 0) {
        const double nr = sqrt(acc);
        nrm64[r] = nr;
        inv32[r] = (float)(1.0 / fmax(nr, 1e-8));
        sq32[r] = (float)acc;
        if (anybad) atomicAdd(nonfinite, 1);
        else atomicMax(xmax_bits, (unsigned long long)__double_as_longlong(nr));
    }
}

hipError_t launch_pack_rows(const float* src, int64_t n, int D, int G, float* X, int64_t row0, double* nrm64,
                            float* inv32, float* sq32, unsigned long long* xmax_bits, int* nonfinite,
                            hipStream_t st) {
    if (n <= 0) return hipSuccess;
    const int64_t blocks = (n + 3) / 4;
    hipLaunchKernelGGL(pack_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, st, src, n, D, G, X, row0, nrm64,
                       inv32, sq32, xmax_bits, nonfinite);
    return hipGetLastError();
}

__global__ void __launch_bounds__(256) unpack_rows_kernel(const float* __restrict__ X, int G, int D, int64_t row0,
                                                          int64_t n, float* __restrict__ dst) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n) return;
    const int lane = threadIdx.x & 63;
    for (int d = lane; d < D; d += 64) dst[row * D + d] = X[tiled_offset((uint64_t)(row0 + row), d, G)];
}

hipError_t launch_unpack_rows(const float* X, int G, int D, int64_t row0, int64_t n, float* dst, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(unpack_rows_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, X, G, D, row0, n, dst);
    return hipGetLastError();
}

// =============================================================================
// Queries
// =============================================================================
__global__ void __launch_bounds__(256) prep_queries_kernel(const float* __restrict__ Q, int B, int D, int G,
                                                           int metric, float* __restrict__ Qt,
                                                           double* __restrict__ qn64) {
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= B) return;
    const int Dp64 = (D + 63) & ~63;
    const float* q = Q + (int64_t)b * D;
    double acc = 0.0;
    for (int d = lane; d < Dp64; d += 64) {
        const double v = d < D ? (double)q[d] : 0.0;
        acc = acc + v * v;
    }
    acc = wave_sum_butterfly(acc);
    const double nq = sqrt(acc);
    if (lane == 0) qn64[b] = nq;
    // cosine: the candidate pass works on q/max(|q|,1e-8) rounded to fp32.
    const float scale = metric == 0 ? (float)(1.0 / fmax(nq, 1e-8)) : 1.0f;
    for (int d = lane; d < D; d += 64) Qt[tiled_offset((uint64_t)b, d, G)] = q[d] * scale;
}

hipError_t launch_prep_queries(const float* Q, int B, int D, int G, int metric, float* Qt, double* qn64,
                               hipStream_t st) {
    hipLaunchKernelGGL(prep_queries_kernel, dim3((B + 3) / 4), dim3(256), 0, st, Q, B, D, G, metric, Qt, qn64);
    return hipGetLastError();
}

// =============================================================================
// Candidate pass: fp32 MFMA scores fused with a per-workgroup top-KP
// =============================================================================
// Workgroup = 4 waves.  Wave w of step s owns row tiles (4 s + w) RT .. +RT-1
// (RT*32 rows) and all QB = 32 QT queries of its query block.  Per 8-dim group
// it issues RT + QT global_load_dwordx4 (corpus from HBM, queries from L2) and
// 4 RT QT v_mfma_f32_32x32x2_f32; loads run P groups ahead in registers (no LDS
// staging: the corpus operand is streamed once and not shared across waves).
// Accumulator lane l / register v holds query 32 qt + (l & 31) against corpus
// row 32 t + (v & 3) + 8 (v >> 2) + 4 (l >> 5).
//
// Top-KP per query lives in LDS: an append buffer of CAP = 2 KP (score, row)
// per query plus a threshold (the KP-th best after the last compaction).  A
// score enters only if it beats the threshold; when a buffer fills, one wave
// bitonic-sorts it and keeps the best KP.  Invariant used by the certificate
// in rerank: every row not in the final list scored <= the list's KP-th entry.
template <int METRIC, int QT, int RT, int KP, int CAP>
__global__ void __launch_bounds__(256, (QT * 32 * CAP * 8 > 80 * 1024) ? 1 : 2)
scan_topk_kernel(const float* __restrict__ X, const float* __restrict__ rowscale, const uint32_t* __restrict__ mask,
                 const float* __restrict__ Qt, int G, int64_t N, int B, int64_t n_steps, int steps_per_wg,
                 float* __restrict__ cand_s, uint32_t* __restrict__ cand_i) {
    constexpr int QB = 32 * QT;
    constexpr int P = 4;
    constexpr int E = CAP / 64;
    __shared__ float s_sc[QB * CAP];
    __shared__ uint32_t s_ix[QB * CAP];
    __shared__ int s_cnt[QB];
    __shared__ float s_thr[QB];

    const int lane = threadIdx.x & 63;
    // wave index made provably uniform: every tile/group address below is then
    // scalar (SGPR base) + lane*16 (one VGPR), keeping VGPRs for the pipeline.
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int n_wg = gridDim.x;
    const int wg = blockIdx.x;
    const int qb = blockIdx.y;
    const int lane4 = lane * 4;

    for (int i = threadIdx.x; i < QB; i += 256) {
        s_cnt[i] = 0;
        s_thr[i] = -INFINITY;
    }
    __syncthreads();

    const int64_t s_begin = (int64_t)wg * steps_per_wg;
    const int64_t s_end = s_begin + steps_per_wg < n_steps ? s_begin + steps_per_wg : n_steps;
    const size_t tstride = (size_t)G * BLOCK_FLOATS;  // floats per row tile
    const float* Qbase = Qt + (size_t)(qb * QT) * tstride;

    // keep a compacted query buffer: sort, keep KP, raise threshold (one wave)
    auto compact = [&](int q) {
        float sv[E];
        uint32_t iv[E];
        const int n = s_cnt[q] < CAP ? s_cnt[q] : CAP;
#pragma unroll
        for (int i = 0; i < E; ++i) {
            const int e = i * 64 + lane;
            sv[i] = e < n ? s_sc[q * CAP + e] : -INFINITY;
            iv[i] = e < n ? s_ix[q * CAP + e] : 0xFFFFFFFFu;
        }
        wave_sort_desc<float, uint32_t, E>(sv, iv);
#pragma unroll
        for (int i = 0; i < E; ++i) {
            const int e = i * 64 + lane;
            if (e < KP) {
                s_sc[q * CAP + e] = sv[i];
                s_ix[q * CAP + e] = iv[i];
            }
        }
        const float th = shfl_t(sv[(KP - 1) >> 6], (KP - 1) & 63);
        if (lane == 0) {
            s_thr[q] = th;
            s_cnt[q] = KP;
        }
    };

    f32x4 xr[P][RT], qr[P][QT];
    if (s_begin < s_end) {
        const float* xs = X + (size_t)((s_begin * 4 + wv) * RT) * tstride;
#pragma unroll
        for (int p = 0; p < P; ++p) {
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
                xr[p][rt] = *(const f32x4*)(xs + rt * tstride + p * BLOCK_FLOATS + lane4);
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
                qr[p][qt] = *(const f32x4*)(Qbase + qt * tstride + p * BLOCK_FLOATS + lane4);
        }
    }

    for (int64_t s = s_begin; s < s_end; ++s) {
        const int64_t t0 = (s * 4 + wv) * RT;
        const float* xs = X + (size_t)t0 * tstride;
        const float* xn = (s + 1 < s_end) ? xs + (size_t)(4 * RT) * tstride : xs;
        f32x16 acc[RT][QT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                for (int v = 0; v < 16; ++v) acc[rt][qt][v] = 0.0f;

        for (int gb = 0; gb < G; gb += P) {
#pragma unroll
            for (int p = 0; p < P; ++p) {
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                        for (int qt = 0; qt < QT; ++qt)
                            acc[rt][qt] = __builtin_amdgcn_mfma_f32_32x32x2f32(xr[p][rt][j], qr[p][qt][j],
                                                                               acc[rt][qt], 0, 0, 0);
                const int gn = gb + p + P;
                const bool cur = gn < G;
                const float* xsrc = cur ? xs + (size_t)gn * BLOCK_FLOATS : xn + (size_t)(gn - G) * BLOCK_FLOATS;
                const float* qsrc = Qbase + (size_t)(cur ? gn : gn - G) * BLOCK_FLOATS;
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) xr[p][rt] = *(const f32x4*)(xsrc + rt * tstride + lane4);
#pragma unroll
                for (int qt = 0; qt < QT; ++qt) qr[p][qt] = *(const f32x4*)(qsrc + qt * tstride + lane4);
            }
        }

        // ---- epilogue: scores, threshold filter, LDS append --------------------
        uint32_t pend[RT][QT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            const int64_t t = t0 + rt;
            const int64_t rb = t * 32 + 4 * (lane >> 5);
            f32x4 rsv[4];
#pragma unroll
            for (int m = 0; m < 4; ++m) rsv[m] = *(const f32x4*)(rowscale + rb + 8 * m);
            const uint32_t mword = mask ? mask[t] : 0xFFFFFFFFu;
#pragma unroll
            for (int qt = 0; qt < QT; ++qt) {
                const int ql = qt * 32 + (lane & 31);
                const bool qvalid = qb * QB + ql < B;
                const float thr = s_thr[ql];
                uint32_t pm = 0;
#pragma unroll
                for (int v = 0; v < 16; ++v) {
                    const int ro = (v & 3) + 8 * (v >> 2) + 4 * (lane >> 5);
                    const float rs = rsv[v >> 2][v & 3];
                    const float a = acc[rt][qt][v];
                    const float sc = METRIC == 0 ? a * rs : fmaf(2.0f, a, -rs);
                    const bool ok = qvalid && (t * 32 + ro < N) && ((mword >> ro) & 1u);
                    acc[rt][qt][v] = sc;
                    if (ok && sc > thr) pm |= 1u << v;
                }
                pend[rt][qt] = pm;
            }
        }

        for (;;) {
            uint32_t left = 0;
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
                for (int qt = 0; qt < QT; ++qt) {
                    if (pend[rt][qt]) {
                        const int ql = qt * 32 + (lane & 31);
#pragma unroll
                        for (int v = 0; v < 16; ++v) {
                            if (pend[rt][qt] & (1u << v)) {
                                const int pos = atomicAdd(&s_cnt[ql], 1);
                                if (pos < CAP) {
                                    const int ro = (v & 3) + 8 * (v >> 2) + 4 * (lane >> 5);
                                    s_sc[ql * CAP + pos] = acc[rt][qt][v];
                                    s_ix[ql * CAP + pos] = (uint32_t)((t0 + rt) * 32 + ro);
                                    pend[rt][qt] &= ~(1u << v);
                                }
                            }
                        }
                    }
                    left |= pend[rt][qt];
                }
            }
            if (!__syncthreads_or(left != 0)) break;
            for (int q = wv; q < QB; q += 4)
                if (s_cnt[q] >= CAP) compact(q);
            __syncthreads();
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
                for (int qt = 0; qt < QT; ++qt) {
                    if (pend[rt][qt]) {
                        const float thr = s_thr[qt * 32 + (lane & 31)];
#pragma unroll
                        for (int v = 0; v < 16; ++v)
                            if (!(acc[rt][qt][v] > thr)) pend[rt][qt] &= ~(1u << v);
                    }
                }
            }
        }
    }

    // ---- flush: sorted top-KP of every query of the block ------------------------
    __syncthreads();
    for (int q = wv; q < QB; q += 4) {
        float sv[E];
        uint32_t iv[E];
        const int n = s_cnt[q] < CAP ? s_cnt[q] : CAP;
#pragma unroll
        for (int i = 0; i < E; ++i) {
            const int e = i * 64 + lane;
            sv[i] = e < n ? s_sc[q * CAP + e] : -INFINITY;
            iv[i] = e < n ? s_ix[q * CAP + e] : 0xFFFFFFFFu;
        }
        wave_sort_desc<float, uint32_t, E>(sv, iv);
        const int qg = qb * QB + q;
        if (qg < B) {
            const size_t base = ((size_t)qg * n_wg + wg) * KP;
#pragma unroll
            for (int i = 0; i < E; ++i) {
                const int e = i * 64 + lane;
                if (e < KP) {
                    cand_s[base + e] = sv[i];
                    cand_i[base + e] = iv[i];
                }
            }
        }
    }
}

template <int METRIC, int QT, int KP, int CAP>
static hipError_t scan_dispatch(const float* X, const float* rowscale, const uint32_t* mask, const float* Qt, int G,
                                int64_t N, int B, int n_qblocks, int64_t n_steps, int n_wg, int spw, float* cs,
                                uint32_t* ci, hipStream_t st) {
    hipLaunchKernelGGL((scan_topk_kernel<METRIC, QT, 2, KP, CAP>), dim3(n_wg, n_qblocks), dim3(256), 0, st, X,
                       rowscale, mask, Qt, G, N, B, n_steps, spw, cs, ci);
    return hipGetLastError();
}

hipError_t launch_scan_topk(int metric, int KP, const float* X, const float* rowscale, const uint32_t* mask,
                            const float* Qt, int G, int64_t N, int B, int n_qblocks, int64_t n_steps, int n_wg,
                            int spw, float* cs, uint32_t* ci, hipStream_t st) {
#define VDB_SCAN(M, QT, KPV)                                                                              \
    if (metric == M && KP == KPV)                                                                         \
        return scan_dispatch<M, QT, KPV, 2 * KPV>(X, rowscale, mask, Qt, G, N, B, n_qblocks, n_steps, n_wg, \
                                                   spw, cs, ci, st);
    VDB_SCAN(0, 2, 32) VDB_SCAN(0, 2, 64) VDB_SCAN(0, 2, 128) VDB_SCAN(0, 1, 256)
    VDB_SCAN(1, 2, 32) VDB_SCAN(1, 2, 64) VDB_SCAN(1, 2, 128) VDB_SCAN(1, 1, 256)
#undef VDB_SCAN
    return hipErrorInvalidValue;
}

// =============================================================================
// Merge of sorted lists (per query, one workgroup)
// =============================================================================
// Each wave folds every 4th list into a running sorted top-KP held in registers
// (bitonic merge of running ++ reversed(new)); lists whose best entry cannot
// enter are skipped after one load.  Waves 1..3 then hand their lists to wave 0
// through LDS.
template <typename K, typename I, int KP>
__global__ void __launch_bounds__(256)
merge_lists_kernel(const K* __restrict__ ls, const I* __restrict__ li, int n_lists, int Lk, int64_t sq, int64_t sj,
                   K* __restrict__ out_k, I* __restrict__ out_i) {
    constexpr int E2 = (2 * KP) / 64;
    __shared__ K s_k[3 * KP];
    __shared__ I s_i[3 * KP];
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int q = blockIdx.x;
    K v[E2];
    I x[E2];
#pragma unroll
    for (int i = 0; i < E2; ++i) {
        v[i] = -INFINITY;
        x[i] = sentinel_idx<I>();
    }
    auto fold = [&](const K* L, const I* Li, int len) {
        const K rw = shfl_t(v[(KP - 1) >> 6], (KP - 1) & 63);
        const I ri = shfl_t(x[(KP - 1) >> 6], (KP - 1) & 63);
        if (len <= 0 || !better(L[0], Li[0], rw, ri)) return;
#pragma unroll
        for (int i = 0; i < E2; ++i) {
            const int e = i * 64 + lane;
            if (e >= KP) {
                const int src = 2 * KP - 1 - e;
                v[i] = src < len ? L[src] : (K)-INFINITY;
                x[i] = src < len ? Li[src] : sentinel_idx<I>();
            }
        }
        wave_merge_desc<K, I, E2>(v, x);
    };
    for (int j = wv; j < n_lists; j += 4) fold(ls + q * sq + j * sj, li + q * sq + j * sj, Lk);
    if (wv > 0) {
#pragma unroll
        for (int i = 0; i < E2; ++i) {
            const int e = i * 64 + lane;
            if (e < KP) {
                s_k[(wv - 1) * KP + e] = v[i];
                s_i[(wv - 1) * KP + e] = x[i];
            }
        }
    }
    __syncthreads();
    if (wv == 0) {
        for (int w = 0; w < 3; ++w) fold(s_k + w * KP, s_i + w * KP, KP);
#pragma unroll
        for (int i = 0; i < E2; ++i) {
            const int e = i * 64 + lane;
            if (e < KP) {
                out_k[(size_t)q * KP + e] = v[i];
                out_i[(size_t)q * KP + e] = x[i];
            }
        }
    }
}

template <typename K, typename I>
static hipError_t merge_dispatch(int KP, const K* lk, const I* li, int n_lists, int Lk, int64_t sq, int64_t sj,
                                 int nq, K* ok, I* oi, hipStream_t st) {
    switch (KP) {
#define VDB_MERGE(KPV)                                                                                       \
    case KPV:                                                                                               \
        hipLaunchKernelGGL((merge_lists_kernel<K, I, KPV>), dim3(nq), dim3(256), 0, st, lk, li, n_lists, Lk, sq, \
                           sj, ok, oi);                                                                     \
        return hipGetLastError();
        VDB_MERGE(32) VDB_MERGE(64) VDB_MERGE(128) VDB_MERGE(256) VDB_MERGE(512) VDB_MERGE(1024)
#undef VDB_MERGE
        default:
            return hipErrorInvalidValue;
    }
}

hipError_t launch_merge_f32(int KP, const float* ls, const uint32_t* li, int n_lists, int B, float* out_s,
                            uint32_t* out_i, hipStream_t st) {
    if (KP > 256) return hipErrorInvalidValue;
    return merge_dispatch<float, uint32_t>(KP, ls, li, n_lists, KP, (int64_t)n_lists * KP, KP, B, out_s, out_i, st);
}

hipError_t launch_merge_f64_u32(int KP, const double* lk, const uint32_t* li, int n_lists, int Lk, int64_t sq,
                                int64_t sj, int nq, double* out_k, uint32_t* out_i, hipStream_t st) {
    return merge_dispatch<double, uint32_t>(KP, lk, li, n_lists, Lk, sq, sj, nq, out_k, out_i, st);
}

hipError_t launch_merge_f64_i64(int KP, const double* lk, const int64_t* li, int n_lists, int Lk, int64_t sq,
                                int64_t sj, int nq, double* out_k, int64_t* out_i, hipStream_t st) {
    return merge_dispatch<double, int64_t>(KP, lk, li, n_lists, Lk, sq, sj, nq, out_k, out_i, st);
}

// =============================================================================
// Exact fp64 keys
// =============================================================================
// key(q, r): cosine  dot / (max(|q|,1e-8) * max(|x|,1e-8))
//            L2      -(sum (x-q)^2)
// in the canonical order (vdb_common.h).  One wave per (query, row).
template <int METRIC>
__device__ __forceinline__ double exact_key(const float* __restrict__ q, double qn, const float* __restrict__ X, int G,
                                            int D, uint64_t r, double xn) {
    const int lane = threadIdx.x & 63;
    const int Dp = (D + 31) & ~31;
    const int Dp64 = (D + 63) & ~63;
    double acc = 0.0;
    for (int d = lane; d < Dp64; d += 64) {
        const double qd = d < D ? (double)q[d] : 0.0;
        const double xd = d < Dp ? (double)X[tiled_offset(r, d, G)] : 0.0;
        if (METRIC == 0) {
            acc = acc + qd * xd;
        } else {
            const double df = xd - qd;
            acc = acc + df * df;
        }
    }
    acc = wave_sum_butterfly(acc);
    if (METRIC == 0) return acc / (fmax(qn, 1e-8) * fmax(xn, 1e-8));
    return -acc;
}

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

// Rerank: exact keys of the KP candidates, best k out, and the certificate that
// the exact top-k lies inside the candidate set:
//   every non-candidate row r has approx a_r <= a_KP (scan invariant), and
//   |approx - exact| <= eps, so if a_KP + eps < a_k - eps no non-candidate can
//   reach the top k.  A failed certificate queues the query for exact_scan.
template <int METRIC, int KP>
__global__ void __launch_bounds__(256) rerank_kernel(RerankArgs a) {
    constexpr int E = KP >= 64 ? KP / 64 : 1;
    __shared__ double s_k[KP];
    __shared__ uint32_t s_i[KP];
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int b = blockIdx.x;
    const float* q = a.Q + (int64_t)b * a.D;
    const double qn = a.qn64[b];
    for (int c = wv; c < KP; c += 4) {
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
        hipLaunchKernelGGL((rerank_kernel<M, KPV>), dim3(B), dim3(256), 0, st, a);           \
        return hipGetLastError();                                                            \
    }
    VDB_RR(0, 32) VDB_RR(0, 64) VDB_RR(0, 128) VDB_RR(0, 256)
    VDB_RR(1, 32) VDB_RR(1, 64) VDB_RR(1, 128) VDB_RR(1, 256)
#undef VDB_RR
    return hipErrorInvalidValue;
}

// Exact scan (certificate fallback, and the path for k > 200): every eligible
// row of a workgroup's range gets its exact key; each wave keeps a private
// sorted top-KE in LDS (append buffer of 2 KE, compacted when full).  Rows are
// visited in increasing order per wave, so a strict '>' against the threshold
// keeps the lower-index-first tie rule.
template <int METRIC, int KE>
__global__ void __launch_bounds__(256)
exact_scan_kernel(const float* __restrict__ Q, const double* __restrict__ qn64, const int* __restrict__ qlist,
                  const float* __restrict__ X, int G, int D, const double* __restrict__ nrm64,
                  const uint32_t* __restrict__ mask, int64_t N, int64_t rows_per_wg, double* __restrict__ lk,
                  uint32_t* __restrict__ li) {
    constexpr int CAP = 2 * KE;
    constexpr int E = CAP / 64;
    constexpr int EK = KE / 64 > 0 ? KE / 64 : 1;
    __shared__ double s_k[4][CAP];
    __shared__ uint32_t s_i[4][CAP];
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int qi = blockIdx.y;
    const int b = qlist ? qlist[qi] : qi;
    const float* q = Q + (int64_t)b * D;
    const double qn = qn64[b];
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_wg;
    const int64_t r1 = r0 + rows_per_wg < N ? r0 + rows_per_wg : N;
    int cnt = 0;
    double thr = -INFINITY;
    auto compact = [&]() {
        double kv[E];
        uint32_t iv[E];
#pragma unroll
        for (int i = 0; i < E; ++i) {
            const int e = i * 64 + lane;
            kv[i] = e < cnt ? s_k[wv][e] : -INFINITY;
            iv[i] = e < cnt ? s_i[wv][e] : 0xFFFFFFFFu;
        }
        wave_sort_desc<double, uint32_t, E>(kv, iv);
#pragma unroll
        for (int i = 0; i < E; ++i) {
            const int e = i * 64 + lane;
            if (e < KE) {
                s_k[wv][e] = kv[i];
                s_i[wv][e] = iv[i];
            }
        }
        thr = shfl_t(kv[(KE - 1) >> 6], (KE - 1) & 63);
        cnt = KE;
    };
    for (int64_t r = r0 + wv; r < r1; r += 4) {
        if (mask && !((mask[r >> 5] >> (r & 31)) & 1u)) continue;
        const double key = exact_key<METRIC>(q, qn, X, G, D, (uint64_t)r, nrm64[r]);
        if (key > thr) {
            if (lane == 0) {
                s_k[wv][cnt] = key;
                s_i[wv][cnt] = (uint32_t)r;
            }
            ++cnt;
            if (cnt == CAP) compact();
        }
    }
    compact();  // sorts what is left; cnt <= CAP
    const int n_lists = gridDim.x * 4;
    const size_t base = ((size_t)qi * n_lists + (size_t)blockIdx.x * 4 + wv) * KE;
#pragma unroll
    for (int i = 0; i < EK; ++i) {
        const int e = i * 64 + lane;
        if (e < KE) {
            lk[base + e] = s_k[wv][e];
            li[base + e] = s_i[wv][e];
        }
    }
}

hipError_t launch_exact_scan(int metric, int KE, const float* Q, const double* qn64, const int* qlist, int nq,
                             const float* X, int G, int D, const double* nrm64, const uint32_t* mask, int64_t N,
                             int n_wg, int64_t rows_per_wg, double* lk, uint32_t* li, hipStream_t st) {
#define VDB_EX(M, KEV)                                                                                        \
    if (metric == M && KE == KEV) {                                                                           \
        hipLaunchKernelGGL((exact_scan_kernel<M, KEV>), dim3(n_wg, nq), dim3(256), 0, st, Q, qn64, qlist, X, G, \
                           D, nrm64, mask, N, rows_per_wg, lk, li);                                           \
        return hipGetLastError();                                                                             \
    }
    VDB_EX(0, 32) VDB_EX(0, 64) VDB_EX(0, 128) VDB_EX(0, 256) VDB_EX(0, 512) VDB_EX(0, 1024)
    VDB_EX(1, 32) VDB_EX(1, 64) VDB_EX(1, 128) VDB_EX(1, 256) VDB_EX(1, 512) VDB_EX(1, 1024)
#undef VDB_EX
    return hipErrorInvalidValue;
}

template <typename I>
__global__ void __launch_bounds__(256) finalize_kernel(int metric, const double* __restrict__ sk,
                                                       const I* __restrict__ si, int KP, int nq,
                                                       const int* __restrict__ qmap, int k, int64_t index_offset,
                                                       float* __restrict__ out_s, int64_t* __restrict__ out_i,
                                                       double* __restrict__ out_k) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= (int64_t)nq * k) return;
    const int qi = (int)(t / k);
    const int e = (int)(t % k);
    const int b = qmap ? qmap[qi] : qi;
    const double key = sk[(size_t)qi * KP + e];
    const I ix = si[(size_t)qi * KP + e];
    const bool valid = sizeof(I) == 8 ? (int64_t)ix >= 0 : (uint32_t)ix != 0xFFFFFFFFu;
    const size_t o = (size_t)b * k + e;
    write_result(metric, key, (uint64_t)ix + (uint64_t)index_offset, valid && key != -INFINITY, out_s + o, out_i + o,
                 out_k ? out_k + o : nullptr);
}

hipError_t launch_finalize_u32(int metric, const double* sk, const uint32_t* si, int KP, int nq, const int* qmap,
                               int k, int64_t index_offset, float* out_s, int64_t* out_i, double* out_k,
                               hipStream_t st) {
    const int64_t n = (int64_t)nq * k;
    hipLaunchKernelGGL(finalize_kernel<uint32_t>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, metric, sk, si,
                       KP, nq, qmap, k, index_offset, out_s, out_i, out_k);
    return hipGetLastError();
}

hipError_t launch_finalize_i64(int metric, const double* sk, const int64_t* si, int KP, int nq, const int* qmap,
                               int k, float* out_s, int64_t* out_i, double* out_k, hipStream_t st) {
    const int64_t n = (int64_t)nq * k;
    hipLaunchKernelGGL(finalize_kernel<int64_t>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, metric, sk, si,
                       KP, nq, qmap, k, (int64_t)0, out_s, out_i, out_k);
    return hipGetLastError();
}

// =============================================================================
// Operator slot: the full score matrix, reference fp32 arithmetic
// =============================================================================
// cosine: x/max(|x|,1e-8) and q/max(|q|,1e-8) in fp32, then the dot product;
// euclidean: sqrt(sum((x-q)^2)).  One wave per corpus row, looping queries; not
// the hot path (service/optimized_vector_store.py:31-48 materialise [N] per
// query, performance/mlx_optimized.py:59-88 [B,N]).
__global__ void __launch_bounds__(256) similarity_matrix_kernel(const float* __restrict__ X, int64_t N, int D,
                                                                const float* __restrict__ Q, int B, int metric,
                                                                float* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= N) return;
    const float* x = X + r * D;
    float xs = 0.0f;
    for (int d = lane; d < D; d += 64) xs = fmaf(x[d], x[d], xs);
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) xs += __shfl_xor(xs, off, 64);
    const float xinv = 1.0f / fmaxf(sqrtf(xs), 1e-8f);
    for (int b = 0; b < B; ++b) {
        const float* q = Q + (int64_t)b * D;
        float acc = 0.0f, qs = 0.0f;
        for (int d = lane; d < D; d += 64) {
            if (metric == 0) {
                acc = fmaf(q[d], x[d] * xinv, acc);
                qs = fmaf(q[d], q[d], qs);
            } else {
                const float df = x[d] - q[d];
                acc = fmaf(df, df, acc);
            }
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            acc += __shfl_xor(acc, off, 64);
            qs += __shfl_xor(qs, off, 64);
        }
        if (lane == 0) out[(int64_t)b * N + r] = metric == 0 ? acc / fmaxf(sqrtf(qs), 1e-8f) : sqrtf(acc);
    }
}

hipError_t launch_similarity_matrix(const float* X, int64_t N, int D, const float* Q, int B, int metric, float* out,
                                    hipStream_t st) {
    if (N <= 0 || B <= 0) return hipSuccess;
    hipLaunchKernelGGL(similarity_matrix_kernel, dim3((unsigned)((N + 3) / 4)), dim3(256), 0, st, X, N, D, Q, B,
                       metric, out);
    return hipGetLastError();
}

}  // namespace vdb
