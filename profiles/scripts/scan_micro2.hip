// scan_micro2.hip — K-loop ablation for the bf16 (hi plane) candidate pass (not product code).
// C2 shape: N = 1M rows, D = 768 (48 groups of 16 dims), B = 64 queries.  The top-k
// epilogue is replaced by a fold of the accumulators.  Variants:
//   QSRC 0: query operand from global memory (L2), prefetched PQ groups ahead in registers
//           (the product kernel's scheme), one 64-query block per workgroup;
//   QSRC 1: the query block of 32 queries (both bf16 planes, 96 KiB) staged ONCE in LDS,
//           read per group with ds_read_b128; B = 64 -> 2 workgroups per row range
//           (XCD-paired, sharing the corpus through L2);
//   CONTIG: 1 = hi plane stored contiguously ([tile4][group][4][64][8] bf16), 0 = the
//           product's split layout (hi and lo 4 KiB planes interleaved; hi read only).
// Build: hipcc --offload-arch=gfx950 -O3 -o scan_micro2 scan_micro2.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
constexpr int BF = 256;  // floats per 1 KiB block

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void stream_read(const f32x4* __restrict__ X, size_t n, float* out) {
    f32x4 acc = {0, 0, 0, 0};
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 7 * stride < n; i += 8 * stride) {
        f32x4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(X + i + u * stride);
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; i < n; i += stride) acc += X[i];
    if (acc[0] == 1234.5f) out[0] = acc[1] + acc[2] + acc[3];
}

template <bool NT>
__device__ __forceinline__ f32x4 ld(const float* p) {
    if constexpr (NT) return __builtin_nontemporal_load((const f32x4*)p);
    else return *(const f32x4*)p;
}

// corpus block address of (row tile t, group g): CONTIG -> hi-only layout, else split layout
template <int CONTIG>
__device__ __forceinline__ size_t cblk(uint64_t t, int g, int G) {
    if constexpr (CONTIG) return (((size_t)(t >> 2) * G + g) * 4 + (t & 3)) * BF;
    return (((size_t)(t >> 2) * G + g) * 8 + (t & 3)) * BF;
}
constexpr size_t PLANE = 4 * BF;  // split layout: lo plane 4 KiB after hi

template <int QSRC, int RT, int QT, int PX, int PQ, int CONTIG, bool NT, int XPL>
__global__ void __launch_bounds__(256, 1) micro(const float* __restrict__ X, const float* __restrict__ Q, int G,
                                                 int spw, int64_t n_steps, int n_qb, float* out) {
    extern __shared__ __attribute__((aligned(16))) float sq[];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane4 = lane * 4;
    // XCD-aware pairing: blocks L and L + 8 j share a row range for j < n_qb
    const int L = blockIdx.x, j = L >> 3;
    const int qb = j % n_qb;
    const int wg = (j / n_qb) * 8 + (L & 7);
    const int64_t s0 = (int64_t)wg * spw;
    const int64_t s1 = s0 + spw < n_steps ? s0 + spw : n_steps;
    // query layout: [qtile][group][plane][64 lanes][8 bf16] = 2 KiB per (qtile, group)
    const float* Qb = Q + (size_t)qb * QT * G * 2 * BF;
    if constexpr (QSRC == 1) {
        for (int e = threadIdx.x; e < QT * G * 2 * BF / 4; e += 256)
            *(f32x4*)(sq + 4 * e) = *(const f32x4*)(Qb + 4 * e);
        __syncthreads();
    }
    f32x4 xr[PX][RT][XPL];
    f32x4 qr[PQ > 0 ? PQ : 1][QT][2];
    float keep = 0.f;
    if (s0 >= s1) return;
    {
        const int64_t t0 = (s0 * 4 + wv) * RT;
#pragma unroll
        for (int p = 0; p < PX; ++p)
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int pl = 0; pl < XPL; ++pl) xr[p][rt][pl] = ld<NT>(X + cblk<CONTIG>(t0 + rt, p, G) + pl * PLANE + lane4);
        if constexpr (QSRC == 0) {
#pragma unroll
            for (int p = 0; p < PQ; ++p)
#pragma unroll
                for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                    for (int pl = 0; pl < 2; ++pl) qr[p][qt][pl] = *(const f32x4*)(Qb + ((size_t)(qt * G + p) * 2 + pl) * BF + lane4);
        }
    }
    for (int64_t s = s0; s < s1; ++s) {
        const int64_t t0 = (s * 4 + wv) * RT;
        const int64_t tn = (s + 1 < s1) ? t0 + 4 * RT : t0;
        f32x16 acc[RT][QT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                for (int v = 0; v < 16; ++v) acc[rt][qt][v] = 0.f;
        for (int gb = 0; gb < G; gb += PX) {
#pragma unroll
            for (int p = 0; p < PX; ++p) {
                const int g = gb + p;
                f32x4 qv[QT][2];
                if constexpr (QSRC == 0) {
#pragma unroll
                    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                        for (int pl = 0; pl < 2; ++pl) qv[qt][pl] = qr[p % PQ][qt][pl];
                } else {
#pragma unroll
                    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                        for (int pl = 0; pl < 2; ++pl) qv[qt][pl] = *(const f32x4*)(sq + ((size_t)(qt * G + g) * 2 + pl) * BF + lane4);
                }
#pragma unroll
                for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                    for (int qt = 0; qt < QT; ++qt) {
                        const bf16x8 xh = __builtin_bit_cast(bf16x8, xr[p][rt][0]);
                        if constexpr (XPL == 2)
                            acc[rt][qt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, xr[p][rt][XPL - 1]), __builtin_bit_cast(bf16x8, qv[qt][0]), acc[rt][qt], 0, 0, 0);
                        acc[rt][qt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xh, __builtin_bit_cast(bf16x8, qv[qt][1]), acc[rt][qt], 0, 0, 0);
                        acc[rt][qt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xh, __builtin_bit_cast(bf16x8, qv[qt][0]), acc[rt][qt], 0, 0, 0);
                    }
                __builtin_amdgcn_sched_barrier(0);
                const int gn = g + PX;
                const bool same = gn < G;
                const int64_t tt = same ? t0 : tn;
                const int gg = same ? gn : gn - G;
#pragma unroll
                for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                    for (int pl = 0; pl < XPL; ++pl) xr[p][rt][pl] = ld<NT>(X + cblk<CONTIG>(tt + rt, gg, G) + pl * PLANE + lane4);
                if constexpr (QSRC == 0) {
                    const int gq = (g + PQ) % G;
#pragma unroll
                    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                        for (int pl = 0; pl < 2; ++pl) qr[p % PQ][qt][pl] = *(const f32x4*)(Qb + ((size_t)(qt * G + gq) * 2 + pl) * BF + lane4);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                for (int v = 0; v < 16; ++v) keep += acc[rt][qt][v];
    }
    if (keep == 1234.5f) out[0] = keep;
}

template <int QSRC, int RT, int QT, int PX, int PQ, int CONTIG, bool NT, int XPL = 1>
void run(const char* name, const float* X, const float* Q, int G, int64_t N, float* out, int n_cu) {
    const int64_t rows_per_step = 4 * RT * 32;
    const int64_t n_steps = (N + rows_per_step - 1) / rows_per_step;
    const int QB = 32 * QT;
    const int n_qb = 64 / QB;
    const int target = n_cu / n_qb;  // one workgroup per CU in total
    const int spw = (int)((n_steps + target - 1) / target);
    const int n_wg = (int)((n_steps + spw - 1) / spw);
    const int n_wg8 = (n_wg + 7) / 8 * 8;
    const size_t lds = QSRC == 1 ? (size_t)QT * G * 2 * 1024 : 0;
    auto k = micro<QSRC, RT, QT, PX, PQ, CONTIG, NT, XPL>;
    if (lds > 64 * 1024) CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k, dim3(n_wg8 * n_qb), dim3(256), lds, 0, X, Q, G, spw, n_steps, n_qb, out);
    CK(hipDeviceSynchronize());
    const int reps = 20;
    CK(hipEventRecord(a));
    for (int w = 0; w < reps; ++w) hipLaunchKernelGGL(k, dim3(n_wg8 * n_qb), dim3(256), lds, 0, X, Q, G, spw, n_steps, n_qb, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    const double bytes = (double)N * G * 16 * 2 * XPL;  // corpus bytes read once per launch
    printf("%-44s %8.1f us  %7.1f GB/s (corpus bytes / time)\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9);
}

int main() {
    const int64_t N = 1 << 20;  // rows (C2 ~ 1M)
    const int G = 48;          // D = 768
    int n_cu = 256;
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    n_cu = p.multiProcessorCount;
    const size_t xfloats = (size_t)N / 32 * G * 2 * BF;  // split layout (2 planes) = 2x the hi plane
    float *X, *Q, *out;
    CK(hipMalloc(&X, xfloats * 4));
    CK(hipMalloc(&Q, (size_t)2 * G * 2 * BF * 4 * 2));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(X, 0, xfloats * 4));
    CK(hipMemset(Q, 0, (size_t)2 * G * 2 * BF * 4 * 2));
    {
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        const size_t n4 = xfloats / 8;  // half the buffer = hi-plane bytes
        hipLaunchKernelGGL(stream_read, dim3(n_cu * 8), dim3(256), 0, 0, (const f32x4*)X, n4, out);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a));
        for (int w = 0; w < 20; ++w) hipLaunchKernelGGL(stream_read, dim3(n_cu * 8), dim3(256), 0, 0, (const f32x4*)X, n4, out);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ms /= 20;
        printf("%-44s %8.1f us  %7.1f GB/s\n", "stream read (nt, 1.6 GB)", ms * 1e3, n4 * 16 / (ms * 1e-3) / 1e9);
        CK(hipEventRecord(a));
        for (int w = 0; w < 20; ++w) hipLaunchKernelGGL(stream_read, dim3(n_cu * 8), dim3(256), 0, 0, (const f32x4*)X, 2 * n4, out);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b));
        ms /= 20;
        printf("%-44s %8.1f us  %7.1f GB/s\n", "stream read (nt, 3.2 GB)", ms * 1e3, 2 * n4 * 16 / (ms * 1e-3) / 1e9);
    }
    // bf16x3 (hi + lo planes, split layout as the product)
    run<0, 2, 2, 4, 4, 0, true, 2>("b3 globalQ RT2 QT2 PX4 PQ4 (product)", X, Q, G, N, out, n_cu);
    run<0, 2, 2, 4, 4, 0, false, 2>("b3 globalQ RT2 QT2 PX4 PQ4 default-policy", X, Q, G, N, out, n_cu);
    run<0, 4, 2, 2, 2, 0, true, 2>("b3 globalQ RT4 QT2 PX2 PQ2", X, Q, G, N, out, n_cu);
    run<0, 4, 2, 3, 3, 0, true, 2>("b3 globalQ RT4 QT2 PX3 PQ3", X, Q, G, N, out, n_cu);
    run<0, 4, 2, 4, 4, 0, true, 2>("b3 globalQ RT4 QT2 PX4 PQ4", X, Q, G, N, out, n_cu);
    run<0, 2, 2, 6, 6, 0, true, 2>("b3 globalQ RT2 QT2 PX6 PQ6", X, Q, G, N, out, n_cu);
    run<1, 2, 1, 8, 0, 0, false, 2>("b3 ldsQ RT2 QT1 PX8", X, Q, G, N, out, n_cu);
    run<1, 4, 1, 4, 0, 0, false, 2>("b3 ldsQ RT4 QT1 PX4", X, Q, G, N, out, n_cu);
    run<1, 4, 1, 6, 0, 0, false, 2>("b3 ldsQ RT4 QT1 PX6", X, Q, G, N, out, n_cu);
    run<1, 4, 1, 6, 0, 0, true, 2>("b3 ldsQ RT4 QT1 PX6 nt", X, Q, G, N, out, n_cu);
    run<1, 8, 1, 3, 0, 0, false, 2>("b3 ldsQ RT8 QT1 PX3", X, Q, G, N, out, n_cu);
    // bf16 hi plane
    run<0, 2, 2, 4, 4, 0, true>("hi globalQ RT2 QT2 PX4 PQ4 split (product)", X, Q, G, N, out, n_cu);
    run<0, 4, 2, 4, 4, 1, true>("hi globalQ RT4 QT2 PX4 PQ4 contig", X, Q, G, N, out, n_cu);
    run<0, 4, 2, 4, 4, 0, true>("hi globalQ RT4 QT2 PX4 PQ4 split", X, Q, G, N, out, n_cu);
    run<0, 4, 2, 6, 6, 1, true>("hi globalQ RT4 QT2 PX6 PQ6 contig", X, Q, G, N, out, n_cu);
    run<1, 8, 1, 6, 0, 1, false>("hi ldsQ RT8 QT1 PX6 contig", X, Q, G, N, out, n_cu);
    run<1, 8, 1, 6, 0, 1, true>("hi ldsQ RT8 QT1 PX6 contig nt", X, Q, G, N, out, n_cu);
    return 0;
}
