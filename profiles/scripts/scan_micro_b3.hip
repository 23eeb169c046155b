// scan_micro_b3.hip — ablation microbenchmark for the bf16x3 candidate-pass K-loop
// (not product code).  Same split-bf16 super-tile layout as vdb_scan.hip; the top-k
// epilogue is replaced by a sum of the accumulators (kept live by one store).
//   stream  : plain grid-stride float4 read of the corpus (HBM read ceiling)
//   MODE 0  : full K-loop (corpus from HBM, queries from L2, 3 MFMA per tile pair)
//   MODE 1  : no query loads (query registers reused)
//   MODE 2  : no MFMA (loads only; the loaded values are xor-folded)
// Build: hipcc --offload-arch=gfx950 -O3 -o scan_micro_b3 scan_micro_b3.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
constexpr int BF = 256;  // floats per 1 KiB block

__global__ void stream_read(const f32x4* __restrict__ X, size_t n, float* out) {
    f32x4 acc = {0, 0, 0, 0};
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 7 * stride < n; i += 8 * stride) {
        f32x4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = X[i + u * stride];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; i < n; i += stride) acc += X[i];
    if (acc[0] == 1234.5f) out[0] = acc[1] + acc[2] + acc[3];
}

template <int MODE, int RT, int QT, int PX, int PQ, int WAVES>
__global__ void __launch_bounds__(64 * WAVES, 1) micro(const float* __restrict__ X, const float* __restrict__ Q, int G,
                                                        int spw, int64_t n_steps, float* out) {
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane4 = lane * 4;
    constexpr size_t GSTEP = 8 * BF, PLANE = 4 * BF;
    auto blk = [](uint64_t t, int g, int GG) -> size_t { return (((size_t)(t >> 2) * GG + g) * 8 + (t & 3)) * BF; };
    const int64_t s0 = (int64_t)blockIdx.x * spw;
    const int64_t s1 = s0 + spw < n_steps ? s0 + spw : n_steps;
    f32x4 xr[PX][RT][2], qr[PQ][QT][2];
    for (int p = 0; p < PX; ++p)
        for (int rt = 0; rt < RT; ++rt)
            for (int pl = 0; pl < 2; ++pl) xr[p][rt][pl] = *(const f32x4*)(X + blk((s0 * WAVES + wv) * RT, p, G) + pl * PLANE + rt * BF + lane4);
    for (int p = 0; p < PQ; ++p)
        for (int qt = 0; qt < QT; ++qt)
            for (int pl = 0; pl < 2; ++pl) qr[p][qt][pl] = *(const f32x4*)(Q + blk(qt, p, G + 8) + pl * PLANE + lane4);
    float keep = 0.f;
    uint32_t kx = 0;
    for (int64_t s = s0; s < s1; ++s) {
        const int64_t t0 = (s * WAVES + wv) * RT;
        const float* xs = X + blk(t0, 0, G);
        const float* xn = (s + 1 < s1) ? X + blk(t0 + WAVES * RT, 0, G) : xs;
        f32x16 acc[RT][QT];
        for (int rt = 0; rt < RT; ++rt)
            for (int qt = 0; qt < QT; ++qt)
                for (int v = 0; v < 16; ++v) acc[rt][qt][v] = 0.f;
        auto group = [&](const int p, const float* xsrc, const float* qsrc) {
            const int pq = p % PQ;
            if (MODE != 2) {
#pragma unroll
                for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                    for (int qt = 0; qt < QT; ++qt) {
                        const bf16x8 xh = __builtin_bit_cast(bf16x8, xr[p][rt][0]), xl = __builtin_bit_cast(bf16x8, xr[p][rt][1]);
                        const bf16x8 qh = __builtin_bit_cast(bf16x8, qr[pq][qt][0]), ql = __builtin_bit_cast(bf16x8, qr[pq][qt][1]);
                        acc[rt][qt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xl, qh, acc[rt][qt], 0, 0, 0);
                        acc[rt][qt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xh, ql, acc[rt][qt], 0, 0, 0);
                        acc[rt][qt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xh, qh, acc[rt][qt], 0, 0, 0);
                    }
            } else {
#pragma unroll
                for (int rt = 0; rt < RT; ++rt)
                    for (int pl = 0; pl < 2; ++pl)
                        for (int j = 0; j < 4; ++j) kx ^= __float_as_uint(xr[p][rt][pl][j]);
#pragma unroll
                for (int qt = 0; qt < QT; ++qt)
                    for (int pl = 0; pl < 2; ++pl)
                        for (int j = 0; j < 4; ++j) kx ^= __float_as_uint(qr[pq][qt][pl][j]);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int pl = 0; pl < 2; ++pl) xr[p][rt][pl] = *(const f32x4*)(xsrc + pl * PLANE + rt * BF + lane4);
            if (MODE != 1) {
#pragma unroll
                for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                    for (int pl = 0; pl < 2; ++pl) qr[pq][qt][pl] = *(const f32x4*)(qsrc + pl * PLANE + qt * BF + lane4);
            }
            __builtin_amdgcn_sched_barrier(0);
        };
        const float* Qb = Q;
        int gb = 0;
        for (; gb < G - PX; gb += PX) {
#pragma unroll
            for (int p = 0; p < PX; ++p) group(p, xs + (size_t)(gb + p + PX) * GSTEP, Qb + (size_t)(gb + p + PQ) * GSTEP);
        }
#pragma unroll
        for (int p = 0; p < PX; ++p) group(p, xn + (size_t)p * GSTEP, Qb + (size_t)(gb + p + PQ) * GSTEP);
        for (int rt = 0; rt < RT; ++rt)
            for (int qt = 0; qt < QT; ++qt)
                for (int v = 0; v < 16; ++v) keep += acc[rt][qt][v];
    }
    out[(size_t)blockIdx.x * blockDim.x + threadIdx.x] = keep + (float)kx;
}

template <int MODE, int RT, int QT, int PX, int PQ, int WAVES>
void run(const char* name, const float* X, const float* Q, int G, int64_t N, int n_wg, float* out, double bytes) {
    const int64_t n_steps = N / (32 * RT * WAVES);
    const int spw = (int)((n_steps + n_wg - 1) / n_wg);
    const int grid = (int)((n_steps + spw - 1) / spw);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL((micro<MODE, RT, QT, PX, PQ, WAVES>), dim3(grid), dim3(64 * WAVES), 0, 0, X, Q, G, spw, n_steps, out);
    hipEventRecord(a);
    const int reps = 10;
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((micro<MODE, RT, QT, PX, PQ, WAVES>), dim3(grid), dim3(64 * WAVES), 0, 0, X, Q, G, spw, n_steps, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    ms /= reps;
    printf("%-34s n_wg %4d grid %4d spw %3d  %.4f ms  %.0f GB/s\n", name, n_wg, grid, spw, ms, bytes / (ms * 1e-3) / 1e9);
}

int main(int argc, char** argv) {
    const int64_t N = 1 << 20;
    const int D = 768, G = D / 16, B = 64;
    float *X, *Q, *out;
    const size_t xbytes = (size_t)N * D * 4;
    hipMalloc(&X, xbytes);
    hipMalloc(&Q, (size_t)128 * (D + 128) * 4);
    hipMalloc(&out, (size_t)8192 * 512 * 4);
    std::vector<uint32_t> h((size_t)N * D);
    for (size_t i = 0; i < h.size(); ++i) h[i] = 0x3F803F80u ^ (uint32_t)((i * 2654435761u) & 0x007F007Fu);
    hipMemcpy(X, h.data(), xbytes, hipMemcpyHostToDevice);
    hipMemcpy(Q, h.data(), (size_t)128 * (D + 128) * 4, hipMemcpyHostToDevice);
    (void)B;
    for (int rep = 0; rep < 2; ++rep) {
        for (int grid : {256, 512, 1024, 2048}) {
            hipEvent_t a, b;
            hipEventCreate(&a);
            hipEventCreate(&b);
            hipLaunchKernelGGL(stream_read, dim3(grid), dim3(256), 0, 0, (const f32x4*)X, xbytes / 16, out);
            hipEventRecord(a);
            for (int r = 0; r < 10; ++r)
                hipLaunchKernelGGL(stream_read, dim3(grid), dim3(256), 0, 0, (const f32x4*)X, xbytes / 16, out);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            ms /= 10;
            printf("stream_read grid %4d  %.4f ms  %.0f GB/s\n", grid, ms, xbytes / (ms * 1e-3) / 1e9);
        }
    }
    run<0, 2, 2, 4, 2, 4>("full RT2 PX4 PQ2 W4", X, Q, G, N, 256, out, xbytes);
    run<0, 2, 2, 4, 4, 4>("full RT2 PX4 PQ4 W4", X, Q, G, N, 256, out, xbytes);
    run<1, 2, 2, 4, 2, 4>("noQ  RT2 PX4 W4", X, Q, G, N, 256, out, xbytes);
    run<2, 2, 2, 4, 2, 4>("noMFMA RT2 PX4 PQ2 W4", X, Q, G, N, 256, out, xbytes);
    run<2, 2, 2, 8, 2, 4>("noMFMA RT2 PX8 PQ2 W4", X, Q, G, N, 256, out, xbytes);
    run<0, 2, 2, 4, 2, 8>("full RT2 PX4 PQ2 W8", X, Q, G, N, 256, out, xbytes);
    run<2, 2, 2, 4, 2, 8>("noMFMA RT2 PX4 PQ2 W8", X, Q, G, N, 256, out, xbytes);
    run<0, 2, 2, 4, 2, 4>("full RT2 PX4 PQ2 W4 x2/CU", X, Q, G, N, 512, out, xbytes);
    run<1, 2, 2, 4, 2, 4>("noQ  RT2 PX4 W4 x2/CU", X, Q, G, N, 512, out, xbytes);
    run<0, 1, 2, 4, 2, 4>("full RT1 PX4 PQ2 W4", X, Q, G, N, 256, out, xbytes);
    run<0, 1, 2, 8, 4, 4>("full RT1 PX8 PQ4 W4", X, Q, G, N, 256, out, xbytes);
    run<0, 1, 2, 4, 2, 8>("full RT1 PX4 PQ2 W8", X, Q, G, N, 256, out, xbytes);
    return 0;
}
