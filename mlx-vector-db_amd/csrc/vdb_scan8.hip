// vdb_scan8.hip — the int8 candidate pass (PREC_I8 / PREC_I8X3, kernel: vdb_scan8_kernel.h):
// the corpus quantisation at ingest, the per-batch query quantisation, the pilot with the same
// arithmetic, and the dispatch to the instantiation units.
#include "vdb_scan8_kernel.h"

// scan_qlds auto (-1): the query block in LDS for short rows (rule 1) and, past 768 dims,
// whenever it fits (rule 2).  Measured (profiles/r04_qlds, same box): C3 (D = 1536) scan 0.625
// -> 0.572 ms with rule 2; C2 (D = 768) 0.153 -> 0.161 ms (slower then: that shape did not load
// the corpus nt, VDB_S8_NTQL).  With nt loads (round 5) C2 runs 0.148 -> 0.143 ms with the block
// in LDS, so rule 2 starts past 16 groups (profiles/r05_ab/ab8_ntql.log).
#ifndef VDB_S8_QLDS_BIG_G8
#define VDB_S8_QLDS_BIG_G8 16
#endif

namespace vdb {

// =============================================================================
// Ingest: the 16-bit fixed-point copy of the centred rows
// =============================================================================
// max |y - mu| over rows [row0, row0 + n) (y = x * inv32 for cosine), as float bits into *out
// (non-negative floats order like their bits): the index's quantisation step s_x derives from it
// at the first add (vdb_api.cpp setup_direction).
__global__ void __launch_bounds__(256) zmax_kernel(const float* __restrict__ X, const float* __restrict__ inv32,
                                                   const float* __restrict__ mu, int64_t row0, int64_t n, int D, int G,
                                                   uint32_t* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    float m = 0.0f;
    if (i < n) {
        const uint64_t r = (uint64_t)(row0 + i);
        const float iv = inv32 ? inv32[r] : 1.0f;
        for (int d = lane; d < D; d += 64) {
            const float x = X[row_piece_offset(r, d >> 2, G) + (d & 3)];
            m = fmaxf(m, fabsf((inv32 ? x * iv : x) - mu[d]));
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
    if (lane == 0 && i < n) atomicMax(out, __float_as_uint(m));
}

hipError_t launch_zmax(const float* X, const float* inv32, const float* mu, int64_t row0, int64_t n, int D, int G,
                       uint32_t* out, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(zmax_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, X, inv32, mu, row0, n, D, G, out);
    return hipGetLastError();
}

// 16 values -> 16 int8 (byte j = element j) in one f32x4
__device__ __forceinline__ f32x4 pack_i8x16(const int (&v)[16]) {
    f32x4 o;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const uint32_t u = (uint32_t)(v[4 * w] & 255) | ((uint32_t)(v[4 * w + 1] & 255) << 8) |
                           ((uint32_t)(v[4 * w + 2] & 255) << 16) | ((uint32_t)(v[4 * w + 3] & 255) << 24);
        o[w] = __uint_as_float(u);
    }
    return o;
}

// t -> (hi, lo) with t ~ hi + lo / 256, |hi|, |lo| <= 127 (values past the range clip; the
// residual the statistics measure then shows it)
__device__ __forceinline__ void split_i8(float t, int& hi, int& lo) {
    hi = (int)fminf(fmaxf(rintf(t), -127.0f), 127.0f);
    lo = (int)fminf(fmaxf(rintf((t - (float)hi) * 256.0f), -127.0f), 127.0f);
}

// One wave per row: z = y - mu, xh / xl planes of the int8 copy (block (tile, 32-dim group g,
// plane) lane i + 32 h holds dims 32 g + 16 h .. + 15 of row 32 t + i), and the row statistics
// (fp64 bits, running maxima) stats[0] |z - s_x xh|, [1] |dir.(z - s_x xh)|, [2] |z - z~|,
// [3] |dir.(z - z~)| (z~ = s_x (xh + xl/256)), [4] |s_x xh|, [5] |s_x xl / 256|.
__global__ void __launch_bounds__(256) quant_rows_kernel(const float* __restrict__ X, const float* __restrict__ inv32,
                                                         const float* __restrict__ mu, const float* __restrict__ dir,
                                                         float sx, int64_t row0, int64_t n, int G,
                                                         float* __restrict__ Xq, unsigned long long* __restrict__ stats,
                                                         int8_t* __restrict__ xh_rm) {
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n) return;
    const uint64_t r = (uint64_t)(row0 + i);
    const float iv = inv32 ? inv32[r] : 1.0f;
    const float isx = 1.0f / sx;
    const int G8 = G >> 2;
    const int nc = 2 * G8;  // 16-dim chunks
    double s_r8 = 0.0, s_d8 = 0.0, s_r16 = 0.0, s_d16 = 0.0, s_h = 0.0, s_l = 0.0;
    for (int c = lane; c < nc; c += 64) {
        const float* src = X + (size_t)r * (size_t)(8 * G) + 16 * c;
        int hv[16], lv[16];
#pragma unroll
        for (int j4 = 0; j4 < 4; ++j4) {
            const f32x4 xv = *(const f32x4*)(src + 4 * j4);
            const f32x4 mv = *(const f32x4*)(mu + 16 * c + 4 * j4);
            const f32x4 dv = *(const f32x4*)(dir + 16 * c + 4 * j4);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float z = (inv32 ? xv[j] * iv : xv[j]) - mv[j];
                int h, l;
                split_i8(z * isx, h, l);
                hv[4 * j4 + j] = h;
                lv[4 * j4 + j] = l;
                const double zh = (double)sx * h, zl = (double)sx * l / 256.0;
                const double r8 = (double)z - zh, r16 = r8 - zl;
                s_r8 += r8 * r8;
                s_r16 += r16 * r16;
                s_d8 += (double)dv[j] * r8;
                s_d16 += (double)dv[j] * r16;
                s_h += zh * zh;
                s_l += zl * zl;
            }
        }
        const uint64_t t = r >> 5;
        float* dst = Xq + corpus_block(t, c >> 1, 0, G8) + (size_t)((r & 31) + 32 * (c & 1)) * 4;
        *(f32x4*)dst = pack_i8x16(hv);
        *(f32x4*)(dst + corpus_plane(G8)) = pack_i8x16(lv);
        // the xh plane row-major too (as xh + 128): the finish's refinement reads candidates' rows whole
        if (xh_rm) {  // biased to unsigned (xh + 128): one v_cvt_f32_ubyte per element in the finish
            int uv[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) uv[j] = hv[j] + 128;
            *(f32x4*)(xh_rm + r * (size_t)(8 * G) + 16 * c) = pack_i8x16(uv);
        }
    }
    s_r8 = wave_sum_butterfly(s_r8);
    s_d8 = wave_sum_butterfly(s_d8);
    s_r16 = wave_sum_butterfly(s_r16);
    s_d16 = wave_sum_butterfly(s_d16);
    s_h = wave_sum_butterfly(s_h);
    s_l = wave_sum_butterfly(s_l);
    if (lane == 0) {
        const double v[6] = {sqrt(s_r8), fabs(s_d8), sqrt(s_r16), fabs(s_d16), sqrt(s_h), sqrt(s_l)};
        bool fin = true;  // a non-finite row (the whole add is rejected) leaves no statistics
#pragma unroll
        for (int k = 0; k < 6; ++k) fin = fin && isfinite(v[k]);
#pragma unroll
        for (int k = 0; k < 6 && fin; ++k) {
            const unsigned long long b = (unsigned long long)__double_as_longlong(v[k]);
            if (b > __atomic_load_n(stats + k, __ATOMIC_RELAXED)) atomicMax(stats + k, b);
        }
    }
}

hipError_t launch_quant_rows(const float* X, const float* inv32, const float* mu, const float* dir, float sx,
                             int64_t row0, int64_t n, int G, float* Xq, unsigned long long* stats, hipStream_t st,
                             int8_t* xh_rm) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(quant_rows_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, X, inv32, mu, dir, sx, row0,
                       n, G, Xq, stats, xh_rm);
    return hipGetLastError();
}

// =============================================================================
// The pass's checksum (ABFT): the integer MFMA sums are exact, so over all rows
// r < N of a query block the accumulators the pass produced must add up (mod 2^32) to
//   sum_r H[r][q] = sum_r rint(rinit[r] / (s_x s_q)) [L2] + sum_d CH[d] qh[q][d]
//   sum_r L[r][q] = sum_d CH[d] ql[q][d] + CL[d] qh[q][d]                        [I8X3]
// with CH / CL the column sums of the int8 copy's planes, kept here at ingest.  A wrong operand
// anywhere in the pass (a stale start value or corpus register, a misindexed tile) moves the sum
// whichever way it moves the row's score -- the under-scoring half included, which the finish's
// approx-vs-exact check (rerank set only) cannot see.
// =============================================================================
// csum[pl * Dp + d] += sum over rows [row0, row0 + n) of plane pl (xh, xl), d < Dp = 32 G8.
// One thread per (plane, 16-dim chunk), kColsumRows rows per workgroup.
constexpr int kColsumRows = 2048;
__global__ void __launch_bounds__(256) colsum8_kernel(const float* __restrict__ Xq, int64_t row0, int64_t n, int G8,
                                                      uint32_t* __restrict__ csum) {
    const int nc = 2 * G8;  // 16-dim chunks per plane
    const int tid = threadIdx.x + blockIdx.y * 256;
    if (tid >= 2 * nc) return;
    const int pl = tid / nc, c = tid - pl * nc;
    const int64_t r0 = row0 + (int64_t)blockIdx.x * kColsumRows;
    const int64_t r1 = min(r0 + (int64_t)kColsumRows, row0 + n);
    int acc[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = 0;
    for (int64_t r = r0; r < r1; ++r) {
        const float* src = Xq + corpus_block((uint64_t)r >> 5, c >> 1, 0, G8) + (size_t)((r & 31) + 32 * (c & 1)) * 4 +
                           (pl ? corpus_plane(G8) : 0);
        const f32x4 v = *(const f32x4*)src;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const uint32_t u = __float_as_uint(v[w]);
#pragma unroll
            for (int bt = 0; bt < 4; ++bt) acc[4 * w + bt] += (int)(int8_t)((u >> (8 * bt)) & 255u);
        }
    }
    if (r0 < r1)
#pragma unroll
        for (int j = 0; j < 16; ++j) atomicAdd(csum + (size_t)pl * 32 * G8 + 16 * c + j, (uint32_t)acc[j]);
}

hipError_t launch_colsum8(const float* Xq, int64_t row0, int64_t n, int G8, uint32_t* csum, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    const int threads = 4 * G8;  // 2 planes x 2 G8 chunks
    hipLaunchKernelGGL(colsum8_kernel, dim3((unsigned)((n + kColsumRows - 1) / kColsumRows), (unsigned)((threads + 255) / 256)),
                       dim3(256), 0, st, Xq, row0, n, G8, csum);
    return hipGetLastError();
}

// The L2 pass's accumulator start values at this batch's scale, rs[r] = rint(rinit[r] * (1 / (s_x
// s_q))) (qscal[2] from prep8; 0 past N), which scan8_kernel loads as its H accumulators' start
// (round 4 converted them in the pass: 16 x (mul, round, convert) per wave-step, with the register
// copies ~20% of C4's vector instructions), and *sum += their sum (mod 2^32), the checksum's term
__global__ void __launch_bounds__(256) rstart8_kernel(const float* __restrict__ rinit, int64_t N, int64_t Np,
                                                      const float* __restrict__ qscal, int* __restrict__ rs,
                                                      uint32_t* __restrict__ out) {
    // 16-byte loads and stores, four in flight per lane (both arrays 16-byte aligned: allocation
    // granularity, Np a multiple of 32); rows N..Np-1 (the last tile's padding) start at 0
    const float invU = qscal[2];
    uint32_t s = 0u;
    const int64_t n4 = Np >> 2, tid = (int64_t)blockIdx.x * 256 + threadIdx.x, nt = (int64_t)gridDim.x * 256;
    const f32x4* r4 = (const f32x4*)rinit;
    i32x4* o4 = (i32x4*)rs;
    auto conv = [&](const f32x4& v, int64_t r) {
        i32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            o[j] = 4 * r + j < N ? __float2int_rn(v[j] * invU) : 0;
            s += (uint32_t)o[j];
        }
        return o;
    };
    int64_t r = tid;
    for (; r + 3 * nt < n4; r += 4 * nt) {
        f32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = r4[r + u * nt];
#pragma unroll
        for (int u = 0; u < 4; ++u) o4[r + u * nt] = conv(v[u], r + u * nt);
    }
    for (; r < n4; r += nt) o4[r] = conv(r4[r], r);
    if (!out) return;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) s += (uint32_t)__shfl_xor((int)s, off, 64);
    // one atomic per workgroup: every one of them goes to the same word, and same-address
    // atomics serialise at the memory side (4 per workgroup over 2048 workgroups: 98 us)
    __shared__ uint32_t s_w[4];
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(out, s_w[0] + s_w[1] + s_w[2] + s_w[3]);
}

hipError_t launch_rstart8(const float* rinit, int64_t N, const float* qscal, int* rs, uint32_t* sum, hipStream_t st) {
    if (N <= 0) return hipSuccess;
    const int64_t Np = (N + 31) / 32 * 32;
    const int64_t blocks = std::min<int64_t>(512, std::max<int64_t>(1, ((Np >> 2) + 1023) / 1024));
    hipLaunchKernelGGL(rstart8_kernel, dim3((unsigned)blocks), dim3(256), 0, st, rinit, N, Np, qscal, rs, sum);
    return hipGetLastError();
}

// TEST ONLY (index knob debug_sink_row8, behind VDB_DEBUG_KNOBS=1): sets both planes of one row of
// the int8 copy to -127 without touching the column sums -- a corpus operand the pass reads wrong
// that UNDER-scores the row for every query with non-negative components (the benchmark's data)
__global__ void __launch_bounds__(64) sink_row8_kernel(float* __restrict__ Xq, int64_t r, int G8) {
    const int nc = 2 * G8;
    const float v = __uint_as_float(0x81818181u);  // four int8 -127
    for (int t = threadIdx.x; t < 2 * nc; t += 64) {
        const int pl = t / nc, c = t - pl * nc;
        float* p = Xq + corpus_block((uint64_t)r >> 5, c >> 1, 0, G8) + (size_t)((r & 31) + 32 * (c & 1)) * 4 +
                   (pl ? corpus_plane(G8) : 0);
        *(f32x4*)p = f32x4{v, v, v, v};
    }
}

hipError_t launch_sink_row8(float* Xq, int64_t row, int G8, hipStream_t st) {
    hipLaunchKernelGGL(sink_row8_kernel, dim3(1), dim3(64), 0, st, Xq, row, G8);
    return hipGetLastError();
}

// =============================================================================
// Queries: one scale per batch, s_q = max |q'| / 127 (q' the fp32 query the other passes use:
// cosine normalised), 16-bit fixed point in two int8 planes, tiles as the split layout
// (s2_blk, G8 + QG_EXTRA groups, the leading ones repeated).  Per query: lsl = the prefilter's
// slack (bound of the L term), qerr = the query's share of the certificate's eps.
// =============================================================================
__global__ void __launch_bounds__(256) prep8_kernel(const float* __restrict__ Q, const double* __restrict__ qn64,
                                                    const float* __restrict__ qmax, int B, int Bp, int D, int G8,
                                                    int metric, int prec, Int8Consts c, float* __restrict__ Qq,
                                                    float* __restrict__ lsl, float* __restrict__ qerr,
                                                    float* __restrict__ qscal, float* __restrict__ qres,
                                                    float* __restrict__ qerr2) {
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= Bp) return;
    float m = 0.0f;
    for (int j = lane; j < B; j += 64) m = fmaxf(m, qmax[j]);
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
    float sq = m > 0.0f ? m / 127.0f : 1.0f;
    // L2: H starts at -|x|^2 / 2 / (s_x s_q), which must stay well inside int32 (with the
    // products' own range): a coarser query scale where it would not (eps follows, qerr)
    if (metric == 1) sq = fmaxf(sq, (float)(c.rmax_half / ((double)c.sx * 1.0e9)));
    const float uH = c.sx * sq;
    if (b == 0 && lane == 0) {
        qscal[0] = uH;
        qscal[1] = uH * (1.0f / 256.0f);
        qscal[2] = 1.0f / uH;
    }
    const bool real = b < B;
    const double nq = real ? qn64[b] : 0.0;
    const float scale = metric == 0 ? (float)(1.0 / fmax(nq, 1e-8)) : 1.0f;
    const float* q = Q + (int64_t)(real ? b : 0) * D;
    const float isq = 1.0f / sq;
    const int GQ = G8 + QG_EXTRA;
    double s_rq = 0.0, s_r8 = 0.0, s_ql = 0.0, s_qh = 0.0;
    for (int cc = lane; cc < 2 * GQ; cc += 64) {
        const int g = cc >> 1, h = cc & 1;
        const int d0 = 32 * (g % G8) + 16 * h;
        int hv[16], lv[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int d = d0 + j;
            const float qv = (real && d < D) ? q[d] * scale : 0.0f;
            split_i8(qv * isq, hv[j], lv[j]);
            if (g < G8) {
                const double qh = (double)sq * hv[j], ql = (double)sq * lv[j] / 256.0;
                const double r8 = (double)qv - qh, rq = r8 - ql;
                s_rq += rq * rq;
                s_r8 += r8 * r8;
                s_ql += ql * ql;
                s_qh += qh * qh;
            }
        }
        float* dst = Qq + s2_blk((uint64_t)(b >> 5), g, GQ) + (size_t)((b & 31) + 32 * h) * 4;
        *(f32x4*)dst = pack_i8x16(hv);
        *(f32x4*)(dst + 4 * BLOCK_FLOATS) = pack_i8x16(lv);
        if (qres && g < G8) {  // I8: the query's rounding residual r = q' - s_q qh, row-major [Bp][8 G8 * 4]
            float* rd = qres + (size_t)b * (size_t)(32 * G8) + d0;
#pragma unroll
            for (int j4 = 0; j4 < 4; ++j4) {
                f32x4 v;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int d = d0 + 4 * j4 + j;
                    const float qv = (real && d < D) ? q[d] * scale : 0.0f;
                    v[j] = qv - sq * (float)hv[4 * j4 + j];
                }
                *(f32x4*)(rd + 4 * j4) = v;
            }
        }
    }
    s_rq = wave_sum_butterfly(s_rq);
    s_r8 = wave_sum_butterfly(s_r8);
    s_ql = wave_sum_butterfly(s_ql);
    s_qh = wave_sum_butterfly(s_qh);
    if (lane == 0) {
        const bool x3 = prec == PREC_I8X3, q16 = x3 || prec == PREC_I8Q;
        const double za = c.zmax_h + (x3 ? c.xl_max : 0.0);  // bound of |z~| (I8 / I8Q: s_x xh alone)
        // I8X3: |L uL| <= |s_x xh| |s_q ql / 256| + |s_x xl / 256| |s_q qh|; I8Q the first term
        // alone (I8 has no L)
        const double sl = q16 ? c.zmax_h * sqrt(s_ql) + (x3 ? c.xl_max * sqrt(s_qh) : 0.0) : 0.0;
        // approx - z.q' = -(z - z~).q' (the corpus term, finish) - z~.(q' - q~) (q~ = s_q qh for
        // I8, s_q (qh + ql / 256) for I8X3 / I8Q) - [I8X3: the dropped s_x s_q xl.ql / 65536]
        // (+ L2: the rounding of H's start, <= 0.5 uH, 1 uH with the fp32 product before it)
        double e = za * sqrt(q16 ? s_rq : s_r8) + (x3 ? c.xl_max * sqrt(s_ql) : 0.0) + (metric == 1 ? (double)uH : 0.0);
        e = 1.01 * (metric == 0 ? e : 2.0 * e);
        lsl[b] = real ? (float)(1.01 * sl) * (1.0f + 1e-5f) + 1e-30f : 0.0f;
        qerr[b] = real ? (float)e * (1.0f + 1e-5f) : 0.0f;
        // with the query rounding corrected per candidate (the finish's refinement, I8): only
        // the L2 start value's rounding is left of the query's share
        if (qerr2) qerr2[b] = real ? (float)(1.01 * (metric == 1 ? 2.0 * (double)uH : 0.0)) * (1.0f + 1e-5f) : 0.0f;
    }
}

hipError_t launch_prep8(const float* Q, const double* qn64, const float* qmax, int B, int Bp, int D, int G8,
                        int metric, int prec, const Int8Consts& c, float* Qq, float* lsl, float* qerr, float* qscal,
                        hipStream_t st, float* qres, float* qerr2) {
    hipLaunchKernelGGL(prep8_kernel, dim3((Bp + 3) / 4), dim3(256), 0, st, Q, qn64, qmax, B, Bp, D, G8, metric, prec, c,
                       Qq, lsl, qerr, qscal, qres, qerr2);
    return hipGetLastError();
}

// =============================================================================
// Pilot (vdb_scan2.hip pilot2 with the int8 arithmetic): best fp32 (half-)score per sampled
// tile and query into the pilot slots; L2 adds the exact fp32 start value per row.
// =============================================================================
constexpr int PILOT8_WAVES = 4;
// waves per sampled tile (each takes every W-th group, partials through LDS): one for short rows
// (C4 / C6) and for long ones (> 24 groups): there the scan's query block leaves < 32 KiB of LDS
// beside it, and an LDS-free pilot runs on the CUs beside another batch's scan instead of after
// it (C3: 411.5 K -> 419-422 K QPS, profiles/r05_ab/ab25_pilot_w1.log; C2's W = 4 pilot fits
// beside its scan: unchanged)
#ifndef VDB_PILOT8_W1
#define VDB_PILOT8_W1 0
#endif
// (wide: the batch's scan is a long-row wide pass, whose 8 waves of 255 registers leave nothing
// beside it, so the pilot only has to be fast alone: four waves per tile, C3 63 -> ~35 us)
__host__ __device__ inline int pilot8_w(int G8, bool wide = false) {
    return VDB_PILOT8_W1 || (G8 > 24 && !wide) ? 1 : G8 >= 16 ? 4 : G8 >= 8 ? 2 : 1;
}

// The checksum's expected values (vdb_scan8_kernel.h), one query per wave of the pilot's first
// B / PILOT8_WAVES workgroups (a dependent load chain each: one workgroup looping over a block's
// 64 queries held the pilot -- and the scan after it -- ~8 us at C6): per query
// sum_d CH[d] qh[d] (+ L: CH ql + CL qh)
template <int PREC>
__device__ __forceinline__ void pilot8_chke(const float* __restrict__ Qq, int G, int B,
                                            const uint32_t* __restrict__ csum, uint32_t* __restrict__ chke) {
    constexpr size_t PLANE = 4 * BLOCK_FLOATS;
    constexpr bool HL = Planes8<PREC>::L;
    const int wv_ = threadIdx.x >> 6, ln = threadIdx.x & 63;
    const int GQ = G + QG_EXTRA, Dp = 32 * G;
    for (int q = blockIdx.x * PILOT8_WAVES + wv_; q < B; q += gridDim.x * PILOT8_WAVES) {
        uint32_t eh = 0u, el = 0u;
        for (int cc = ln; cc < 2 * G; cc += 64) {
            const int g = cc >> 1, h = cc & 1, d0 = 32 * g + 16 * h;
            const float* src = Qq + s2_blk((uint64_t)(q >> 5), g, GQ) + (size_t)((q & 31) + 32 * h) * 4;
            const f32x4 qh4 = *(const f32x4*)src;
            const f32x4 ql4 = *(const f32x4*)(src + PLANE);
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const uint32_t uh = __float_as_uint(qh4[w]), ul = __float_as_uint(ql4[w]);
#pragma unroll
                for (int bt = 0; bt < 4; ++bt) {
                    const int d = d0 + 4 * w + bt;
                    const uint32_t hv = (uint32_t)(int)(int8_t)((uh >> (8 * bt)) & 255u);
                    const uint32_t ch = csum[d];
                    eh += hv * ch;
                    if (HL) el += (uint32_t)(int)(int8_t)((ul >> (8 * bt)) & 255u) * ch + (PREC == PREC_I8X3 ? hv * csum[Dp + d] : 0u);
                }
            }
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            eh += (uint32_t)__shfl_xor((int)eh, off, 64);
            el += (uint32_t)__shfl_xor((int)el, off, 64);
        }
        if (ln == 0) {
            chke[2 * (size_t)q] = eh;
            chke[2 * (size_t)q + 1] = el;
        }
    }
}

template <int PREC, int METRIC, int QT>
__global__ void __launch_bounds__(64 * PILOT8_WAVES)
pilot8_scores_kernel(const float* __restrict__ Xq, const float* __restrict__ rinit, const uint32_t* __restrict__ mask,
                     const float* __restrict__ Qq, const float* __restrict__ qscal, int G, int64_t N, int B, int n_qb,
                     int64_t n_tiles, int n_sample, uint32_t* __restrict__ pslots,
                     const uint32_t* __restrict__ csum, uint32_t* __restrict__ chke, int W) {
    constexpr int QB = 32 * QT;
    constexpr int XPL = Planes8<PREC>::XPL;
    constexpr size_t GSTEP = 8 * BLOCK_FLOATS, PLANE = 4 * BLOCK_FLOATS;
    constexpr bool HL = Planes8<PREC>::L;
    if (chke) pilot8_chke<PREC>(Qq, G, B, csum, chke);
    // the group partials of waves part > 0 (W > 1 only: dynamic, so a one-wave-per-tile launch
    // holds no LDS and keeps 8 workgroups per CU; I8: 32 KiB, I8X3 64)
    extern __shared__ int s_pdyn[];
    typedef int PartT[HL ? 2 : 1][QT][16][64];
    PartT* s_part = (PartT*)s_pdyn;
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int part = wv % W;
    const int i = blockIdx.x * (PILOT8_WAVES / W) + wv / W;
    const bool live = i < n_sample;
    const uint64_t t = live ? (uint64_t)((int64_t)i * n_tiles / n_sample) : 0;
    const float* xs = Xq + corpus_block(t, 0, 0, G) + lane * 4;
    const size_t XGSTEP = corpus_gstep(), XPLANE = corpus_plane(G);
    const float uH = qscal[0], uL = qscal[1];
    const uint32_t valid = live ? tile_valid16(mask, (int64_t)t, N, lane) : 0u;
    float rr[16];
#pragma unroll
    for (int v = 0; v < 16; ++v)
        rr[v] = METRIC == 1 && live && part == 0 ? rinit[t * 32 + (v & 3) + 8 * (v >> 2) + 4 * (lane >> 5)] : 0.0f;
    // Every query block of the batch against this wave's sampled tile: the tile and its start
    // values are read once (round 4 ran one workgroup per (tile, query block): C4's 8 blocks read
    // each sampled tile 8 times over 16 K workgroups, 219 us per batch with one stream)
    for (int qb = 0; qb < n_qb; ++qb) {
        const float* qs = Qq + s2_blk((uint64_t)(qb * QT), 0, G + QG_EXTRA) + lane * 4;
        i32x16 aH[1][QT], aL[1][QT];
#pragma unroll
        for (int qt = 0; qt < QT; ++qt)
#pragma unroll
            for (int v = 0; v < 16; ++v) aH[0][qt][v] = aL[0][qt][v] = 0;
        // the wave's groups PC at a time: every load of a chunk issued before its first MFMA
#ifndef VDB_PILOT8_PC
#define VDB_PILOT8_PC 4
#endif
        constexpr int PC = VDB_PILOT8_PC;
        for (int g0 = part; g0 < G; g0 += W * PC) {
            constexpr int QPL = Planes8<PREC>::QPL;
            f32x4 xr[PC][1][XPL], qr[PC][QT][QPL];
#pragma unroll
            for (int j = 0; j < PC; ++j) {
                const int g = g0 + W * j < G ? g0 + W * j : g0;
#pragma unroll
                for (int pl = 0; pl < XPL; ++pl) xr[j][0][pl] = *(const f32x4*)(xs + g * XGSTEP + pl * XPLANE);
#pragma unroll
                for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                    for (int pl = 0; pl < QPL; ++pl)
                        qr[j][qt][pl] = *(const f32x4*)(qs + g * GSTEP + pl * PLANE + qt * BLOCK_FLOATS);
            }
#pragma unroll
            for (int j = 0; j < PC; ++j)
                if (g0 + W * j < G) group_mfma8<PREC, 1, QT>(xr[j], qr[j], aH, aL);
        }
        if (W > 1) {  // (W is uniform over the workgroup: every wave reaches both barriers)
            if (part > 0) {
#pragma unroll
                for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                    for (int v = 0; v < 16; ++v) {
                        s_part[wv][0][qt][v][lane] = aH[0][qt][v];
                        if constexpr (HL) s_part[wv][HL ? 1 : 0][qt][v][lane] = aL[0][qt][v];
                    }
            }
            __syncthreads();
            if (part == 0)
                for (int w = 1; w < W; ++w)
#pragma unroll
                    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                        for (int v = 0; v < 16; ++v) {
                            aH[0][qt][v] += s_part[wv + w][0][qt][v][lane];
                            if constexpr (HL) aL[0][qt][v] += s_part[wv + w][HL ? 1 : 0][qt][v][lane];
                        }
            __syncthreads();
        }
        if (part > 0 || !live) continue;
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
            const int q = qb * QB + qt * 32 + (lane & 31);
            float best = -INFINITY;
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                const float sv = fmaf((float)aH[0][qt][v], uH, (float)aL[0][qt][v] * uL) + rr[v];
                best = ((valid >> v) & 1u) ? fmaxf(best, sv) : best;
            }
            if (METRIC == 1) best = 2.0f * best;
            best = fmaxf(best, __shfl_xor(best, 32, 64));  // the tile's two row halves (lane, lane + 32)
            if (lane < 32 && q < B && best != -INFINITY)
                atomicMax(pslots + pslot_at(q, i % PILOT_SLOTS, B), order_key(best));
        }
    }
}

// Short rows (4 groups of 32 dims, D <= 128: C4 / C6): one wave per sampled tile holds the tile
// in registers, and the next query block's tiles are loaded while the current block's MFMAs and
// epilogue run (the generic loop waited for every block's loads: C4, 4096 tiles x 8 blocks,
// 116 us with one stream, ~10x its MFMA time) -- a cheaper pilot affords a larger sample, whose
// bound then spares the scan more insertions (C4, 16 K tiles: scan 2.32 -> 2.11 ms)
template <int PREC, int METRIC, int QT>
__global__ void __launch_bounds__(64 * PILOT8_WAVES)
pilot8_g4_kernel(const float* __restrict__ Xq, const float* __restrict__ rinit, const uint32_t* __restrict__ mask,
                 const float* __restrict__ Qq, const float* __restrict__ qscal, int64_t N, int B, int n_qb,
                 int64_t n_tiles, int n_sample, uint32_t* __restrict__ pslots, const uint32_t* __restrict__ csum,
                 uint32_t* __restrict__ chke) {
    constexpr int G = 4, QB = 32 * QT;
    constexpr int XPL = Planes8<PREC>::XPL, QPL = Planes8<PREC>::QPL;
    constexpr size_t GSTEP = 8 * BLOCK_FLOATS, PLANE = 4 * BLOCK_FLOATS;
    if (chke) pilot8_chke<PREC>(Qq, G, B, csum, chke);
    const int lane = threadIdx.x & 63;
    const int i = blockIdx.x * PILOT8_WAVES + (threadIdx.x >> 6);
    if (i >= n_sample) return;  // (no barriers below)
    const uint64_t t = (uint64_t)((int64_t)i * n_tiles / n_sample);
    const float* xs = Xq + corpus_block(t, 0, 0, G) + lane * 4;
    const size_t XGSTEP = corpus_gstep(), XPLANE = corpus_plane(G);
    f32x4 xr[G][1][XPL];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int pl = 0; pl < XPL; ++pl) xr[g][0][pl] = *(const f32x4*)(xs + g * XGSTEP + pl * XPLANE);
    float rr[16];
    if constexpr (METRIC == 1) {
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            const f32x4 r4 = *(const f32x4*)(rinit + t * 32 + 8 * a + 4 * (lane >> 5));
#pragma unroll
            for (int b = 0; b < 4; ++b) rr[4 * a + b] = r4[b];
        }
    } else {
#pragma unroll
        for (int v = 0; v < 16; ++v) rr[v] = 0.0f;
    }
    const uint32_t valid = tile_valid16(mask, (int64_t)t, N, lane);
    const float uH = qscal[0], uL = qscal[1];
    auto load_q = [&](int qb, f32x4 (&q)[G][QT][QPL]) {
        const float* qs = Qq + s2_blk((uint64_t)(qb * QT), 0, G + QG_EXTRA) + lane * 4;
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                for (int pl = 0; pl < QPL; ++pl) q[g][qt][pl] = *(const f32x4*)(qs + g * GSTEP + pl * PLANE + qt * BLOCK_FLOATS);
    };
    f32x4 qa[G][QT][QPL], qn[G][QT][QPL];
    load_q(0, qa);
    for (int qb = 0; qb < n_qb; ++qb) {
        if (qb + 1 < n_qb) load_q(qb + 1, qn);
        i32x16 aH[1][QT], aL[1][QT];
#pragma unroll
        for (int qt = 0; qt < QT; ++qt)
#pragma unroll
            for (int v = 0; v < 16; ++v) aH[0][qt][v] = aL[0][qt][v] = 0;
#pragma unroll
        for (int g = 0; g < G; ++g) group_mfma8<PREC, 1, QT>(xr[g], qa[g], aH, aL);
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
            const int q = qb * QB + qt * 32 + (lane & 31);
            float best = -INFINITY;
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                const float sv = fmaf((float)aH[0][qt][v], uH, (float)aL[0][qt][v] * uL) + rr[v];
                best = ((valid >> v) & 1u) ? fmaxf(best, sv) : best;
            }
            if (METRIC == 1) best = 2.0f * best;
            best = fmaxf(best, __shfl_xor(best, 32, 64));  // the tile's two row halves (lane, lane + 32)
            if (lane < 32 && q < B && best != -INFINITY)
                atomicMax(pslots + pslot_at(q, i % PILOT_SLOTS, B), order_key(best));
        }
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                for (int pl = 0; pl < QPL; ++pl) qa[g][qt][pl] = qn[g][qt][pl];
    }
}

hipError_t launch_pilot8(int prec, int metric, const float* Xq, const float* rinit, const uint32_t* mask,
                         const float* Qq, const float* qscal, int G8, int64_t N, int B, int n_qblocks, int QB,
                         int n_sample, uint32_t* pslots, hipStream_t st, const uint32_t* csum, uint32_t* chke,
                         bool wide) {
    const int64_t n_tiles = (N + 31) / 32;
    const int W = pilot8_w(G8, wide);
    if (n_sample > n_tiles) n_sample = (int)n_tiles;
    if (n_sample <= 0) return hipSuccess;
    const int tpb = G8 == 4 ? PILOT8_WAVES : PILOT8_WAVES / W;
    // (with the checksum's expectations: at least B / PILOT8_WAVES workgroups, one query per wave;
    // past n_sample they score nothing)
    const int gx = (n_sample + tpb - 1) / tpb;
    const dim3 grid(chke ? std::max(gx, (B + PILOT8_WAVES - 1) / PILOT8_WAVES) : gx);
    bool launched = false;
#define VDB_PILOT8(P, M, QTV)                                                                                    \
    if (!launched && prec == P && metric == M && QB == 32 * QTV && G8 == 4) {                                    \
        hipLaunchKernelGGL((pilot8_g4_kernel<P, M, QTV>), grid, dim3(64 * PILOT8_WAVES), 0, st, Xq, rinit, mask, Qq, \
                           qscal, N, B, n_qblocks, n_tiles, n_sample, pslots, csum, chke);                      \
        launched = true;                                                                                         \
    }                                                                                                            \
    if (!launched && prec == P && metric == M && QB == 32 * QTV) {                                               \
        const size_t lds = W > 1 ? (size_t)PILOT8_WAVES * (P == PREC_I8 ? 1 : 2) * QTV * 16 * 64 * 4 : 0;            \
        hipLaunchKernelGGL((pilot8_scores_kernel<P, M, QTV>), grid, dim3(64 * PILOT8_WAVES), lds, st, Xq, rinit, \
                           mask, Qq, qscal, G8, N, B, n_qblocks, n_tiles, n_sample, pslots, csum, chke, W);     \
        launched = true;                                                                                         \
    }
    VDB_PILOT8(PREC_I8, 0, 2) VDB_PILOT8(PREC_I8, 1, 2) VDB_PILOT8(PREC_I8, 0, 1) VDB_PILOT8(PREC_I8, 1, 1)
    VDB_PILOT8(PREC_I8X3, 0, 2) VDB_PILOT8(PREC_I8X3, 1, 2) VDB_PILOT8(PREC_I8X3, 0, 1) VDB_PILOT8(PREC_I8X3, 1, 1)
    VDB_PILOT8(PREC_I8Q, 0, 2) VDB_PILOT8(PREC_I8Q, 1, 2) VDB_PILOT8(PREC_I8Q, 0, 1) VDB_PILOT8(PREC_I8Q, 1, 1)
#undef VDB_PILOT8
    if (!launched) return hipErrorInvalidValue;
    return hipGetLastError();
}

// =============================================================================
// Dispatch
// =============================================================================
int scan8_rows_per_step(int prec, int metric) { return scan8_rows(prec, metric); }

hipError_t launch_scan8(int prec, int metric, int KP, const float* Xq, const float* rinit, const uint32_t* mask,
                        const float* Qq, const float* lsl, const float* qscal, int G8, int64_t N, int B,
                        int n_qblocks, int64_t n_steps, int n_wg, int spw, float* gl_s, uint32_t* gl_i,
                        uint32_t* gl_cnt, int64_t gl_cap, uint32_t* gthr,
                        int lockstep, int qlds, hipStream_t st, const int* gate, uint32_t* chkp, int chk_ld, int chk_l) {
    // the query block in LDS (scan8_qlds): qlds 1 = the round-3 rule (short rows), 2 = whenever
    // it fits, -1 = auto (rule 2 past VDB_S8_QLDS_BIG_G8 groups), 0 = never -- except for rows of fewer 32-dim groups
    // than the global-operand variants keep in flight (PX = 4)
    const int mode = qlds < 0 ? (G8 > VDB_S8_QLDS_BIG_G8 ? 2 : 1) : qlds;
    const bool ql = (mode != 0 && scan8_qlds(G8, KP, prec, metric, mode == 1)) || G8 < 4;
    const bool fs = !lockstep;
    const bool nt = (!ql || (VDB_S8_NTQL && fs)) && n_qblocks == 1;
    auto* unit = prec == PREC_I8X3 ? (metric == 0 ? launch_scan8_i3c : launch_scan8_i3l)
                 : prec == PREC_I8 ? (metric == 0 ? launch_scan8_i1c : launch_scan8_i1l)
                 : prec == PREC_I8Q ? (metric == 0 ? launch_scan8_iqc : launch_scan8_iql)
                                   : nullptr;
    if (!unit || metric < 0 || metric > 1) return hipErrorInvalidValue;
    return unit(KP, Xq, rinit, mask, Qq, lsl, qscal, G8, N, B, n_qblocks, n_steps, n_wg, spw, gl_s, gl_i, gl_cnt,
                gl_cap, gthr, nt, ql, fs, gate, chkp, chk_ld, chk_l, st);
}

}  // namespace vdb
