// scan_micro.hip — ablation microbenchmark for the candidate-pass inner loop
// (not product code).  Same tiling as vdb_scan.hip's K-loop, with the top-k
// epilogue replaced by one store per lane, in modes:
//   0 full loop (corpus from HBM, queries from L2)
//   1 corpus window wraps inside 2 MiB (L2-resident corpus)
//   2 no query loads (registers reused)
//   3 no corpus loads (registers reused)
//   4 no loads at all (MFMA only)
//   5 full loop + a per-step threshold pass over every score and two barriers
// Build: hipcc --offload-arch=gfx950 -O3 -o scan_micro scan_micro.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int MODE, int RT, int QT, int P>
__global__ void __launch_bounds__(256, 2) micro(const float* __restrict__ X, const float* __restrict__ Q, int G,
                                                int steps_per_wg, int64_t n_steps, float* out) {
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane4 = lane * 4;
    const size_t tstride = (size_t)G * 256;
    const int64_t s0 = (int64_t)blockIdx.x * steps_per_wg;
    const int64_t s1 = s0 + steps_per_wg < n_steps ? s0 + steps_per_wg : n_steps;
    const size_t wrap = (2u << 20) / 4;  // floats
    f32x4 xr[P][RT], qr[P][QT];
    for (int p = 0; p < P; ++p) {
        for (int rt = 0; rt < RT; ++rt) xr[p][rt] = *(const f32x4*)(X + rt * tstride + p * 256 + lane4);
        for (int qt = 0; qt < QT; ++qt) qr[p][qt] = *(const f32x4*)(Q + qt * tstride + p * 256 + lane4);
    }
    float keep = 0.f;
    __shared__ float s_thr[64];
    __shared__ int s_cnt;
    if (threadIdx.x < 64) s_thr[threadIdx.x] = 1e30f;
    __syncthreads();
    for (int64_t s = s0; s < s1; ++s) {
        const int64_t t0 = (s * 4 + wv) * RT;
        size_t xoff = (size_t)t0 * tstride;
        if (MODE == 1) xoff %= wrap;
        const float* xs = X + xoff;
        f32x16 acc[RT][QT];
        for (int rt = 0; rt < RT; ++rt)
            for (int qt = 0; qt < QT; ++qt)
                for (int v = 0; v < 16; ++v) acc[rt][qt][v] = 0.f;
        auto group = [&](const int p, const float* xsrc, const float* qsrc) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                    for (int qt = 0; qt < QT; ++qt)
                        acc[rt][qt] = __builtin_amdgcn_mfma_f32_32x32x2f32(xr[p][rt][j], qr[p][qt][j], acc[rt][qt], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            if (MODE != 3 && MODE != 4) {
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) xr[p][rt] = *(const f32x4*)(xsrc + rt * tstride + lane4);
            }
            if (MODE != 2 && MODE != 4) {
#pragma unroll
                for (int qt = 0; qt < QT; ++qt) qr[p][qt] = *(const f32x4*)(qsrc + qt * tstride + lane4);
            }
            __builtin_amdgcn_sched_barrier(0);
        };
        int gb = 0;
        for (; gb < G - P; gb += P) {
#pragma unroll
            for (int p = 0; p < P; ++p) group(p, xs + (size_t)(gb + p + P) * 256, Q + (size_t)(gb + p + P) * 256);
        }
#pragma unroll
        for (int p = 0; p < P; ++p) group(p, xs + (size_t)(p) * 256, Q + (size_t)p * 256);
        if (MODE == 5) {
            // per-step top-k-like epilogue: threshold compare of every score + 2 barriers
            __syncthreads();
            float thr = s_thr[lane & 63];
            int cnt = 0;
            for (int rt = 0; rt < RT; ++rt)
                for (int qt = 0; qt < QT; ++qt)
                    for (int v = 0; v < 16; ++v) cnt += acc[rt][qt][v] > thr ? 1 : 0;
            if (cnt > 1000) atomicAdd(&s_cnt, cnt);
            __syncthreads();
        }
        for (int rt = 0; rt < RT; ++rt)
            for (int qt = 0; qt < QT; ++qt)
                for (int v = 0; v < 16; ++v) keep += acc[rt][qt][v];
    }
    out[(size_t)blockIdx.x * 256 + threadIdx.x] = keep;
}

template <int MODE>
float run(const float* X, const float* Q, int G, int64_t N, int n_wg, float* out) {
    const int64_t n_steps = N / 256;
    const int spw = (int)((n_steps + n_wg - 1) / n_wg);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL((micro<MODE, 2, 2, 4>), dim3(n_wg), dim3(256), 0, 0, X, Q, G, spw, n_steps, out);
    hipEventRecord(a);
    const int reps = 10;
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((micro<MODE, 2, 2, 4>), dim3(n_wg), dim3(256), 0, 0, X, Q, G, spw, n_steps, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

int main(int argc, char** argv) {
    const int64_t N = 1 << 20;
    const int D = 768, G = D / 8, B = 64;
    const int n_wg = argc > 1 ? atoi(argv[1]) : 512;
    float *X, *Q, *out;
    hipMalloc(&X, (size_t)N * D * 4);
    hipMalloc(&Q, (size_t)B * D * 4);
    hipMalloc(&out, (size_t)8192 * 256 * 4);
    std::vector<float> h((size_t)N * D);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.f;
    hipMemcpy(X, h.data(), (size_t)N * D * 4, hipMemcpyHostToDevice);
    hipMemcpy(Q, h.data(), (size_t)B * D * 4, hipMemcpyHostToDevice);
    const double flops = 2.0 * B * N * D;
    float t[6];
    t[0] = run<0>(X, Q, G, N, n_wg, out);
    t[1] = run<1>(X, Q, G, N, n_wg, out);
    t[2] = run<2>(X, Q, G, N, n_wg, out);
    t[3] = run<3>(X, Q, G, N, n_wg, out);
    t[4] = run<4>(X, Q, G, N, n_wg, out);
    t[5] = run<5>(X, Q, G, N, n_wg, out);
    const char* names[6] = {"full", "corpus-in-L2", "no-query-loads", "no-corpus-loads", "mfma-only", "full+epilogue"};
    for (int m = 0; m < 6; ++m)
        printf("n_wg=%d mode %d %-16s %.3f ms  %.1f TF/s\n", n_wg, m, names[m], t[m], flops / (t[m] * 1e-3) / 1e12);
    return 0;
}
