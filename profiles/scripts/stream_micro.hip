// stream_micro.hip — the int8 pass's corpus stream alone (no MFMA, no epilogue): what the memory
// system gives this access pattern.  Layout as the int8 copy: [super tile][group][plane][4 KiB]
// (a super tile = 128 rows, a group = 32 dims, a plane = 4 sub tiles x 1 KiB).  One 256-thread
// workgroup per CU (XCD-interleaved as the scan), each wave streams its own super tile of each
// step: G groups x RT (= 4) KiB of plane 0 (I8) or both planes (I8X3), PX groups in flight.
// Variants: plane 0 only vs both planes; plane-major (the hi planes of a super tile contiguous);
// a rotated start per workgroup (phase).  Timing: hipEvents over R launches.
// Build: hipcc -O3 --offload-arch=gfx950 stream_micro.hip -o stream_micro
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int PX, int PL, bool PM, int G>
__global__ void __launch_bounds__(256, 1) stream_kernel(const float* __restrict__ X, long n_st, int spw,
                                                        int rot, float* __restrict__ sink) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int L = blockIdx.x;
    const int wg = (L >> 3) * 8 + (L & 7);
    const long s0 = (long)wg * spw;
    const long s1 = s0 + spw < n_st ? s0 + spw : n_st;
    if (s0 >= s1) return;
    const long nst = s1 - s0;
    const long srot = rot ? (long)(wg * 7919) % nst : 0;  // rotated start step
    f32x4 acc = {0, 0, 0, 0};
    f32x4 xr[PX][4][PL];
    // block of (super tile st, group g, plane pl, sub tile u) in floats (256 per 1 KiB block)
    auto blk = [&](long st, int g, int pl, int u) -> long {
        if (PM) return (((st * 2 + pl) * G + g) * 4 + u) * 256L;
        return (((st * G + g) * 2 + pl) * 4 + u) * 256L;
    };
    const long total = nst * G;  // group index over this wave's sequence
    auto src = [&](long i, int pl, int u) -> const float* {
        long k = i / G;
        const int g = (int)(i % G);
        k = (k + srot) % nst;
        const long st = (s0 + k) * 4 + wv;  // the wave's super tile of step k
        return X + blk(st, g, pl, u) + lane * 4;
    };
#pragma unroll
    for (int p = 0; p < PX; ++p)
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int pl = 0; pl < PL; ++pl) xr[p][u][pl] = *(const f32x4*)src(p, pl, u);
    for (long i = 0; i < total; i += PX) {
#pragma unroll
        for (int p = 0; p < PX; ++p) {
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int pl = 0; pl < PL; ++pl) acc += xr[p][u][pl];
            const long nx = i + p + PX < total ? i + p + PX : i + p;
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int pl = 0; pl < PL; ++pl) xr[p][u][pl] = *(const f32x4*)src(nx, pl, u);
        }
    }
    if (acc[0] + acc[1] + acc[2] + acc[3] == 12345.0f) sink[threadIdx.x] = acc[0];
}

template <int PX, int PL, bool PM, int G>
static void run(const char* name, const float* X, long n_st, int ncu, int rot, float* sink, double bytes) {
    const int n_wg = ncu;
    const int spw = (int)((n_st + n_wg - 1) / n_wg);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int w = 0; w < 3; ++w) stream_kernel<PX, PL, PM, G><<<(n_wg + 7) / 8 * 8, 256>>>(X, n_st, spw, rot, sink);
    (void)hipEventRecord(a);
    const int R = 20;
    for (int r = 0; r < R; ++r) stream_kernel<PX, PL, PM, G><<<(n_wg + 7) / 8 * 8, 256>>>(X, n_st, spw, rot, sink);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    ms /= R;
    printf("%-34s G %2d PX %d planes %d rot %d: %8.1f us  %6.2f TB/s\n", name, G, PX, PL, rot, ms * 1e3,
           bytes / (ms * 1e-3) / 1e12);
}

int main(int argc, char** argv) {
    const long rows = argc > 1 ? atol(argv[1]) : 10000000;
    const int D = argc > 2 ? atoi(argv[2]) : 128;
    const int G = D / 32;
    const long n_st = (rows + 511) / 512;  // steps of 512 rows (4 waves x 128)
    const long st_tot = n_st * 4;
    const size_t fl = (size_t)st_tot * G * 2 * 4 * 256;
    float* X = nullptr;
    float* sink = nullptr;
    if (hipMalloc(&X, fl * 4) != hipSuccess || hipMalloc(&sink, 4096) != hipSuccess) return 1;
    (void)hipMemset(X, 1, fl * 4);
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    const int ncu = prop.multiProcessorCount;
    const double b1 = (double)st_tot * G * 4096, b2 = 2 * b1;
    printf("rows %ld D %d (%ld steps, %d CUs); plane-0 bytes %.2f GB\n", rows, D, n_st, ncu, b1 / 1e9);
    if (G == 4) {
        run<2, 1, false, 4>("plane 0 (I8), group-major", X, n_st, ncu, 0, sink, b1);
        run<4, 1, false, 4>("plane 0 (I8), group-major", X, n_st, ncu, 0, sink, b1);
        run<8, 1, false, 4>("plane 0 (I8), group-major", X, n_st, ncu, 0, sink, b1);
        run<4, 1, false, 4>("plane 0 (I8), group-major", X, n_st, ncu, 1, sink, b1);
        run<4, 1, true, 4>("plane 0 (I8), plane-major", X, n_st, ncu, 0, sink, b1);
        run<8, 1, true, 4>("plane 0 (I8), plane-major", X, n_st, ncu, 0, sink, b1);
        run<2, 2, false, 4>("both planes, group-major", X, n_st, ncu, 0, sink, b2);
        run<4, 2, false, 4>("both planes, group-major", X, n_st, ncu, 0, sink, b2);
    } else {
        run<2, 1, false, 24>("plane 0 (I8), group-major", X, n_st, ncu, 0, sink, b1);
        run<4, 1, false, 24>("plane 0 (I8), group-major", X, n_st, ncu, 0, sink, b1);
        run<8, 1, false, 24>("plane 0 (I8), group-major", X, n_st, ncu, 0, sink, b1);
        run<4, 1, true, 24>("plane 0 (I8), plane-major", X, n_st, ncu, 0, sink, b1);
        run<4, 2, false, 24>("both planes, group-major", X, n_st, ncu, 0, sink, b2);
    }
    (void)hipFree(X);
    return 0;
}
