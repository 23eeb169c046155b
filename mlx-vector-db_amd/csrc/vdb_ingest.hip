// vdb_ingest.hip: ingest (pack/unpack) and query preparation — part of the gfx950 kernels of the brute-force distance + top-k path
// (pipeline overview: vdb_scan.hip).  Built with -ffp-contract=off.
#include "vdb_common.h"
#include "vdb_internal.h"

namespace vdb {

// =============================================================================
// Ingest
// =============================================================================
// One wave per row.  Canonical fp64 norm (vdb_common.h), row-major store of whole
// 16-byte pieces (padding dims of the row are written as zeros), the fp32 row terms of
// the candidate passes, and (second pass over the row, cache-hot) the bf16 rounding
// residual of the row the split copy holds (cosine: x * inv32, the normalised row; L2: x),
// which bounds the PREC_BF16 certificate.
__global__ void __launch_bounds__(256) pack_rows_kernel(const float* __restrict__ src, int64_t n, int D, int G,
                                                        float* __restrict__ X, int64_t row0,
                                                        double* __restrict__ nrm64, float* __restrict__ inv32,
                                                        float* __restrict__ sq32, float* __restrict__ rinit32,
                                                        int normalise, unsigned long long* __restrict__ xmax_bits,
                                                        int* __restrict__ nonfinite) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n) return;
    const int Dp = G * GROUP_DIMS;
    const int np = (D + 255) / 256;
    const float* s = src + row * (int64_t)D;
    const uint64_t r = (uint64_t)(row0 + row);
    double acc = 0.0;
    int bad = 0;
    for (int m = 0; m < np; ++m) {
        const int p = m * 64 + lane;
        f32x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int d = 4 * p + j;
            v[j] = d < D ? s[d] : 0.0f;
            bad |= !isfinite(v[j]);
            const double dv = (double)v[j];
            acc = acc + dv * dv;
        }
        if (4 * p < Dp) *(f32x4*)(X + row_piece_offset(r, p, G)) = v;
    }
    acc = wave_sum_butterfly(acc);
    const double nr = sqrt(acc);
    const float iv = (float)(1.0 / fmax(nr, 1e-8));
    // the split copy's row and its bf16 residual |y - bf16(y)|
    double res = 0.0, yy = 0.0;
    for (int m = 0; m < np; ++m) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int d = 4 * (m * 64 + lane) + j;
            const float x = d < D ? s[d] : 0.0f;
            const float y = normalise ? x * iv : x;
            const double rv = (double)y - (double)__uint_as_float(bf16_rne_bits(y) << 16);
            res = res + rv * rv;
            yy = yy + (double)y * (double)y;
        }
    }
    res = wave_sum_butterfly(res);
    yy = wave_sum_butterfly(yy);
    const int anybad = __any(bad);
    if (lane == 0) {
        nrm64[r] = nr;
        inv32[r] = iv;
        sq32[r] = (float)acc;
        rinit32[r] = -0.5f * (float)acc;
        if (anybad) {
            atomicAdd(nonfinite, 1);
        } else {
            // xmax_bits[0] max |x|; [1] max |y - bf16(y)| / max(|y|, 1e-8); [2] max |y - bf16(y)|
            // (non-negative doubles order like their bit patterns; a plain read first: the
            // maxima are monotone, so a stale value only lets an atomic through)
            const double dr = sqrt(res);
            const unsigned long long v[3] = {(unsigned long long)__double_as_longlong(nr),
                                             (unsigned long long)__double_as_longlong(dr / fmax(sqrt(yy), 1e-8)),
                                             (unsigned long long)__double_as_longlong(dr)};
#pragma unroll
            for (int i = 0; i < 3; ++i)
                if (v[i] > __atomic_load_n(xmax_bits + i, __ATOMIC_RELAXED)) atomicMax(xmax_bits + i, v[i]);
        }
    }
}

hipError_t launch_pack_rows(const float* src, int64_t n, int D, int G, float* X, int64_t row0, double* nrm64,
                            float* inv32, float* sq32, float* rinit32, int normalise, unsigned long long* xmax_bits,
                            int* nonfinite, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    const int64_t blocks = (n + 3) / 4;
    hipLaunchKernelGGL(pack_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, st, src, n, D, G, X, row0, nrm64,
                       inv32, sq32, rinit32, normalise, xmax_bits, nonfinite);
    return hipGetLastError();
}

// Direction of the bf16 residual bound (PREC_BF16): column sums of the split
// copy's rows y (cosine: x / |x| rounded as the split rounds it) over rows [row0, row0 + n).
// Block: 64 rows; thread d0: dims d0, d0 + 256, ...; fp64 partial sums, one atomic per dim.
__global__ void __launch_bounds__(256) dir_sum_kernel(const float* __restrict__ X, const float* __restrict__ inv32,
                                                      int64_t row0, int64_t n, int D, int G,
                                                      double* __restrict__ sums) {
    const int64_t r0 = (int64_t)blockIdx.x * 64;
    const int64_t r1 = r0 + 64 < n ? r0 + 64 : n;
    for (int d = threadIdx.x; d < D; d += 256) {
        double acc = 0.0;
        for (int64_t i = r0; i < r1; ++i) {
            const uint64_t r = (uint64_t)(row0 + i);
            const float x = X[row_piece_offset(r, d >> 2, G) + (d & 3)];
            acc += (double)(inv32 ? x * inv32[r] : x);
        }
        atomicAdd(sums + d, acc);
    }
}

hipError_t launch_dir_sum(const float* X, const float* inv32, int64_t row0, int64_t n, int D, int G, double* sums,
                          hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(dir_sum_kernel, dim3((unsigned)((n + 63) / 64)), dim3(256), 0, st, X, inv32, row0, n, D, G,
                       sums);
    return hipGetLastError();
}

// |dir . (y - bf16(y))| per row (one wave per row), maximum into *out (fp64 bits): with
// R = max |y - bf16(y)| (pack_rows) and M = this maximum, a query q scores every row's
// bf16 copy within |q - c dir| R + |c| M, c = q . dir (finish_kernel) -- a fraction of
// Cauchy-Schwarz's |q| R when the rows share a mean direction (uniform data: ~0.6).
__global__ void __launch_bounds__(256) resid_dir_kernel(const float* __restrict__ X, const float* __restrict__ inv32,
                                                        int64_t row0, int64_t n, int D, int G,
                                                        const float* __restrict__ dir,
                                                        unsigned long long* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n) return;
    const uint64_t r = (uint64_t)(row0 + i);
    const float iv = inv32 ? inv32[r] : 1.0f;
    const int np = (D + 255) / 256;
    double acc = 0.0;
    for (int m = 0; m < np; ++m) {
        const int p = m * 64 + lane;
        if (4 * p >= D) break;
        const f32x4 xv = *(const f32x4*)(X + row_piece_offset(r, p, G));
        const f32x4 dv = *(const f32x4*)(dir + 4 * p);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float y = inv32 ? xv[j] * iv : xv[j];
            const double rv = (double)y - (double)__uint_as_float(bf16_rne_bits(y) << 16);
            acc = acc + (double)dv[j] * rv;
        }
    }
    acc = wave_sum_butterfly(acc);
    if (lane == 0) {
        const unsigned long long v = (unsigned long long)__double_as_longlong(fabs(acc));
        if (v > __atomic_load_n(out, __ATOMIC_RELAXED)) atomicMax(out, v);
    }
}

hipError_t launch_resid_dir(const float* X, const float* inv32, int64_t row0, int64_t n, int D, int G,
                            const float* dir, unsigned long long* out, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(resid_dir_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, X, inv32, row0, n, D, G, dir,
                       out);
    return hipGetLastError();
}

// Row-major fp32 rows -> split-bf16 tiles.  Thread (tile t, fp32 group g8, row-in-tile i):
// the 8 dims 8 g8 .. 8 g8 + 7 of row 32 t + i (32 contiguous bytes), times inv32[row] for
// cosine (the normalised row the candidate pass scores), -> lane i + 32 (g8 & 1) of the hi
// and lo blocks of 16-dim group g8 >> 1.  A block's 256 threads cover 8 groups of one
// tile: 32 rows x 256 contiguous bytes read, 512 B runs written.
__global__ void __launch_bounds__(256) split_rows_kernel(const float* __restrict__ X, int G, int64_t t0,
                                                         int64_t n_tiles, const float* __restrict__ inv32,
                                                         float* __restrict__ Xs) {
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= n_tiles * G * 32) return;
    const int i = (int)(idx & 31);
    const int g8 = (int)((idx >> 5) % G);
    const uint64_t t = (uint64_t)(t0 + (idx >> 5) / G);
    const float* src = X + row_piece_offset(t * 32 + i, 2 * g8, G);
    f32x4 a = *(const f32x4*)src;
    f32x4 b = *(const f32x4*)(src + 4);
    if (inv32) {
        const float iv = inv32[t * 32 + i];
        a *= iv;
        b *= iv;
    }
    f32x4 hi, lo;
    split8(a, b, hi, lo);
    float* dst = Xs + corpus_block(t, g8 >> 1, 0, G >> 1) + (size_t)(i + 32 * (g8 & 1)) * 4;
    *(f32x4*)dst = hi;
    *(f32x4*)(dst + corpus_plane(G >> 1)) = lo;
}

hipError_t launch_split_rows(const float* X, int G, int64_t row0, int64_t n, const float* inv32, float* Xs,
                             hipStream_t st) {
    if (n <= 0) return hipSuccess;
    const int64_t t0 = row0 >> 5, t1 = (row0 + n + 31) >> 5;
    const int64_t total = (t1 - t0) * G * 32;
    hipLaunchKernelGGL(split_rows_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, X, G, t0, t1 - t0,
                       inv32, Xs);
    return hipGetLastError();
}

// Row-major fp32 rows -> fp32 tiles (the PREC_FP32 candidate copy), whole row tiles
// covering [row0, row0 + n).  Thread (tile t, piece p, row-in-tile i).
__global__ void __launch_bounds__(256) tile_rows_kernel(const float* __restrict__ X, int G, int64_t t0,
                                                        int64_t n_tiles, float* __restrict__ Xt) {
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= n_tiles * 2 * G * 32) return;
    const int i = (int)(idx & 31);
    const int p = (int)((idx >> 5) % (2 * G));
    const uint64_t r = (uint64_t)(t0 + (idx >> 5) / (2 * G)) * 32 + i;
    *(f32x4*)(Xt + tiled_piece_offset(r, p, G)) = *(const f32x4*)(X + row_piece_offset(r, p, G));
}

hipError_t launch_tile_rows(const float* X, int G, int64_t row0, int64_t n, float* Xt, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    const int64_t t0 = row0 >> 5, t1 = (row0 + n + 31) >> 5;
    const int64_t total = (t1 - t0) * 2 * G * 32;
    hipLaunchKernelGGL(tile_rows_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, X, G, t0, t1 - t0,
                       Xt);
    return hipGetLastError();
}

__global__ void __launch_bounds__(256) unpack_rows_kernel(const float* __restrict__ X, int G, int D, int64_t row0,
                                                          int64_t n, float* __restrict__ dst) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n) return;
    const int lane = threadIdx.x & 63;
    for (int d = lane; d < D; d += 64) dst[row * D + d] = X[(size_t)(row0 + row) * (size_t)(8 * G) + d];
}

hipError_t launch_unpack_rows(const float* X, int G, int D, int64_t row0, int64_t n, float* dst, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(unpack_rows_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, X, G, D, row0, n, dst);
    return hipGetLastError();
}

// =============================================================================
// Queries
// =============================================================================
// One wave per padded query slot: canonical fp64 norm, tiled (cosine:
// pre-normalised in fp32) query block including its zero padding, and the
// certificate counter reset (one fewer memset per search).
__global__ void __launch_bounds__(256) prep_queries_kernel(const float* __restrict__ Q, int B, int Bp, int D, int G,
                                                           int metric, float* __restrict__ Qt, float* __restrict__ Qs,
                                                           double* __restrict__ qn64, int* __restrict__ flag_count,
                                                           uint32_t* __restrict__ gthr,
                                                           uint32_t* __restrict__ gslots, uint32_t* __restrict__ gl_cnt,
                                                           int* __restrict__ done, float* __restrict__ qmax,
                                                           const float* __restrict__ mu,
                                                           const float* __restrict__ dir,
                                                           double* __restrict__ qconst) {
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b == 0 && lane == 0 && flag_count) {
        flag_count[0] = 0;      // certificate failures (list follows)
        flag_count[B + 1] = 0;  // of which: candidate-list overflows
        flag_count[B + 2] = 0;  // of which: the finish's approx-vs-exact consistency guard
    }
    if (b >= Bp) return;
    if (lane == 0 && gthr) gthr[b] = 0u;
    if (lane == 0 && gl_cnt) gl_cnt[b] = 0u;
    if (lane == 0 && done) done[b] = 0;
    if (gslots)  // [Bp][KP_MAX] publish slots, then the pilot slots (pslot_at: slot-major over B)
        for (int j = lane; j < KP_MAX + PILOT_SLOTS; j += 64)
            gslots[j < KP_MAX ? (size_t)b * KP_MAX + j : (size_t)Bp * KP_MAX + pslot_at(b, j - KP_MAX, B)] = 0u;
    const int Dp = G * GROUP_DIMS;
    const int np = (D + 255) / 256;
    const bool real = b < B;
    const float* q = Q + (int64_t)(real ? b : 0) * D;
    double acc = 0.0;
    for (int m = 0; m < np; ++m) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int d = 4 * (m * 64 + lane) + j;
            const double v = (real && d < D) ? (double)q[d] : 0.0;
            acc = acc + v * v;
        }
    }
    acc = wave_sum_butterfly(acc);
    const double nq = sqrt(acc);
    if (lane == 0) qn64[b] = nq;
    // cosine: the candidate pass works on q/max(|q|,1e-8) rounded to fp32.
    const float scale = metric == 0 ? (float)(1.0 / fmax(nq, 1e-8)) : 1.0f;
    if (qconst) {
        // the finish's per-query constants (vdb_exact.hip finish_kernel): mu.q' (the int8 pass's
        // shift) and, for the directional corpus bound, c = dir.q' and |q' - c dir|^2 =
        // |q'|^2 - 2 c^2 + c^2 |dir|^2 (fp64; one pass of float4 loads, all in flight together)
        const double qs = metric == 0 ? 1.0 / fmax(nq, 1e-8) : 1.0;
        double mq = 0.0, c = 0.0, q2 = 0.0, d2 = 0.0;
        for (int m = 0; m < np; ++m) {
            const int d0 = 4 * (m * 64 + lane);
            f32x4 qv = {0.f, 0.f, 0.f, 0.f}, mv = {0.f, 0.f, 0.f, 0.f}, dv = {0.f, 0.f, 0.f, 0.f};
            if (d0 < Dp) {  // mu / dir are [Dp], zero padded; the query row is [D]
#pragma unroll
                for (int j = 0; j < 4; ++j) qv[j] = (real && d0 + j < D) ? q[d0 + j] : 0.0f;
                if (mu) mv = *(const f32x4*)(mu + d0);
                if (dir) dv = *(const f32x4*)(dir + d0);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const double x = (double)qv[j] * qs;
                mq += x * (double)mv[j];
                c += x * (double)dv[j];
                q2 += x * x;
                d2 += (double)dv[j] * (double)dv[j];
            }
        }
        mq = wave_sum_butterfly(mq);
        c = wave_sum_butterfly(c);
        q2 = wave_sum_butterfly(q2);
        d2 = wave_sum_butterfly(d2);
        if (lane == 0) {
            qconst[3 * (size_t)b] = mu ? mq : 0.0;
            qconst[3 * (size_t)b + 1] = dir ? c : 0.0;
            qconst[3 * (size_t)b + 2] = dir ? fmax(q2 - 2.0 * c * c + c * c * d2, 0.0) : 0.0;
        }
    }
    if (qmax && real) {  // the int8 pass's batch scale (vdb_scan8.hip prep8)
        float m = 0.0f;
        for (int d = lane; d < D; d += 64) m = fmaxf(m, fabsf(q[d] * scale));
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
        if (lane == 0) qmax[b] = m;
    }
    if (Qt) {
        const int GQ = G + QG_EXTRA;
        for (int p = lane; 4 * p < Dp + 8 * QG_EXTRA; p += 64) {
            const int ps = 4 * p < Dp ? p : p - 2 * G;  // source piece (duplicated groups wrap)
            f32x4 v;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int d = 4 * ps + j;
                v[j] = (real && d < D) ? q[d] * scale : 0.0f;
            }
            *(f32x4*)(Qt + tiled_piece_offset((uint64_t)b, p, GQ)) = v;
        }
    }
    if (Qs) {
        // split-bf16 query tile: half-group h8 = 8 dims; 16-dim groups G/2 + QG_EXTRA, the
        // trailing QG_EXTRA groups repeat the leading ones (modulo G/2)
        const int G16 = G >> 1, GQ16 = G16 + QG_EXTRA;
        for (int h8 = lane; h8 < 2 * GQ16; h8 += 64) {
            const int g16 = h8 >> 1, h = h8 & 1;
            const int d0 = 16 * (g16 % G16) + 8 * h;
            f32x4 a, c;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                a[j] = (real && d0 + j < D) ? q[d0 + j] * scale : 0.0f;
                c[j] = (real && d0 + 4 + j < D) ? q[d0 + 4 + j] * scale : 0.0f;
            }
            f32x4 hi, lo;
            split8(a, c, hi, lo);
            float* dst = Qs + split_block((uint64_t)(b >> 5), g16, GQ16) + (size_t)((b & 31) + 32 * h) * 4;
            *(f32x4*)dst = hi;
            *(f32x4*)(dst + 4 * BLOCK_FLOATS) = lo;
        }
    }
}

hipError_t launch_prep_queries(const float* Q, int B, int Bp, int D, int G, int metric, float* Qt, float* Qs,
                               double* qn64, int* flag_count, uint32_t* gthr, uint32_t* gslots, uint32_t* gl_cnt,
                               int* done, hipStream_t st, float* qmax, const float* mu, const float* dir,
                               double* qconst) {
    hipLaunchKernelGGL(prep_queries_kernel, dim3((Bp + 3) / 4), dim3(256), 0, st, Q, B, Bp, D, G, metric, Qt, Qs,
                       qn64, flag_count, gthr, gslots, gl_cnt, done, qmax, mu, dir, qconst);
    return hipGetLastError();
}
}  // namespace vdb
