// mfma_rate.hip — cycles per MFMA on one SIMD (one wave per SIMD, every CU), the shapes the
// candidate passes use: v_mfma_i32_32x32x32_i8 (int8 pass) vs v_mfma_f32_32x32x16_bf16 (split
// pass), 8 independent accumulators (the passes' 4 x 2 tiles), operands in VGPRs / AGPRs as
// the compiler places them.  s_memtime around the loop (shader cycles).
// Build: hipcc -O3 --offload-arch=gfx950 mfma_rate.hip -o mfma_rate
#include <hip/hip_runtime.h>
#include <cstdio>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int KIND>
__global__ void __launch_bounds__(256, 1) rate_kernel(const int* __restrict__ in, int iters, unsigned long long* out,
                                                      int* sink) {
    const int lane = threadIdx.x & 63;
    i32x4 a[4], b[2];
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = i32x4{in[lane + i], in[lane + 4 + i], in[lane + 8 + i], in[lane + 12 + i]};
#pragma unroll
    for (int i = 0; i < 2; ++i) b[i] = i32x4{in[lane + 16 + i], in[lane + 20 + i], in[lane + 24 + i], in[lane + 28 + i]};
    i32x16 ai[4][2];
    f32x16 af[4][2];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                ai[r][q][v] = 0;
                af[r][q][v] = 0.0f;
            }
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                if constexpr (KIND == 0)
                    ai[r][q] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[r], b[q], ai[r][q], 0, 0, 0);
                else
                    af[r][q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a[r]),
                                                                       __builtin_bit_cast(bf16x8, b[q]), af[r][q], 0, 0, 0);
            }
    }
    int s = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < 2; ++q) s += KIND == 0 ? ai[r][q][lane & 15] : (int)af[r][q][lane & 15];
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();  // after the results are read
    if (s == 0x7fffffff) sink[0] = s;
    if (lane == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

int main() {
    int* in = nullptr;
    int* sink = nullptr;
    unsigned long long* out = nullptr;
    (void)hipMalloc(&in, 4096 * 4);
    (void)hipMalloc(&sink, 64);
    (void)hipMalloc(&out, 256 * 4 * 8);
    (void)hipMemset(in, 1, 4096 * 4);
    const int iters = 4096;
    for (int kind = 0; kind < 2; ++kind) {
        for (int rep = 0; rep < 2; ++rep) {
            if (kind == 0) rate_kernel<0><<<256, 256>>>(in, iters, out, sink);
            else rate_kernel<1><<<256, 256>>>(in, iters, out, sink);
            (void)hipDeviceSynchronize();
        }
        unsigned long long h[1024];
        (void)hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
        double m = 0;
        for (int i = 0; i < 1024; ++i) m += (double)h[i];
        m /= 1024;
        printf("%s: %.1f cycles per MFMA (8 accumulators, %d iterations, every CU)\n",
               kind == 0 ? "v_mfma_i32_32x32x32_i8  " : "v_mfma_f32_32x32x16_bf16", m / (iters * 8.0), iters);
    }
    return 0;
}
