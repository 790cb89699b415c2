// Dependent-issue latency probe for the ops on the Viterbi step's chain
// (one wave, one SIMD): fp64 add, fp64 max, a quad-broadcast DPP move
// followed by an fp64 add, and four independent add chains interleaved.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/lat_probe tools/lat_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int N = 512;

__device__ __forceinline__ double bcast0(double v)
{
    const int lo = __builtin_amdgcn_mov_dpp((int)__double2loint(v), 0x00, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)__double2hiint(v), 0x00, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}

template <int MODE>
__global__ void __launch_bounds__(64) probe(const double *in, double *out, long long *cyc)
{
    double x = in[threadIdx.x], y = in[64 + threadIdx.x];
    double x1 = x + 1.0, x2 = x + 2.0, x3 = x + 3.0;
    const long long t0 = wall_clock64();
    const long long c0 = clock64();
#pragma unroll
    for (int i = 0; i < N; ++i) {
        if constexpr (MODE == 0) {
            x = x + y;
            __asm__ volatile("" : "+v"(x));
        } else if constexpr (MODE == 1) {
            x = fmax(x, y);
            __asm__ volatile("" : "+v"(x));
        } else if constexpr (MODE == 2) {
            x = bcast0(x) + y;
        } else if constexpr (MODE == 4) {
            const double c = x + y;
            x = fmax(c, y);
            __asm__ volatile("" : "+v"(x));
        } else {
            x = x + y;
            x1 = x1 + y;
            x2 = x2 + y;
            x3 = x3 + y;
        }
    }
    const long long c1 = clock64();
    const long long t1 = wall_clock64();
    out[threadIdx.x] = x + x1 + x2 + x3;
    if (threadIdx.x == 0) {
        cyc[0] = c1 - c0;
        cyc[1] = t1 - t0;
    }
}

template <int MODE>
static void run(const char *name, const double *din, double *dout, long long *dcyc)
{
    long long h[2];
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(probe<MODE>, dim3(1), dim3(64), 0, 0, din, dout, dcyc);
        (void)hipDeviceSynchronize();
    }
    (void)hipMemcpy(h, dcyc, sizeof(h), hipMemcpyDeviceToHost);
    int rate = 0;
    (void)hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, 0);
    printf("%-28s clock64 %.2f per op, wall %.2f ns per op (wall clock %d kHz)\n", name, (double)h[0] / N,
           (double)h[1] * 1e6 / rate / N, rate);
}

int main()
{
    double hin[128];
    for (int i = 0; i < 128; ++i)
        hin[i] = 1.0 + 1e-3 * i;
    double *din, *dout;
    long long *dcyc;
    (void)hipMalloc(&din, sizeof(hin));
    (void)hipMalloc(&dout, 64 * sizeof(double));
    (void)hipMalloc(&dcyc, 2 * sizeof(long long));
    (void)hipMemcpy(din, hin, sizeof(hin), hipMemcpyHostToDevice);
    run<0>("dependent v_add_f64", din, dout, dcyc);
    run<1>("dependent v_max_f64", din, dout, dcyc);
    run<2>("dpp bcast + v_add_f64", din, dout, dcyc);
    run<3>("4 chains of v_add_f64 (x4)", din, dout, dcyc);
    run<4>("v_add_f64 -> v_max_f64", din, dout, dcyc);
    return 0;
}
