// Probe of the gfx950 fp64 matrix instructions (tools only, not the product):
//  1. operand maps of v_mfma_f64_4x4x4_16b_f64: which lanes of A and B feed
//     which lane of D (A / B lanes set to distinct powers of two, the other
//     operand to 1: every D entry decodes to the set of lanes it summed);
//  2. issue rate of v_mfma_f64_16x16x4_f64 against v_mfma_f64_4x4x4_16b_f64
//     (both 2048 FLOP per wave instruction): many waves, 8 independent
//     accumulators each, a long loop, timed with HIP events.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/mfma_probe tools/mfma_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void map_kernel(int which, int half, double *out)
{
    const int l = threadIdx.x;
    const bool mine = (l >> 5) == half;
    const double bit = mine ? (double)(1ull << (l & 31)) : 0.0;
    const double a = which == 0 ? bit : 1.0;
    const double b = which == 0 ? 1.0 : bit;
    const double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
    out[l] = d;
}

template <int KIND>
__global__ void __launch_bounds__(256) rate_kernel(double *sink, int iters)
{
    const double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
    if constexpr (KIND == 0) {
        d4 acc[8];
#pragma unroll
        for (int i = 0; i < 8; ++i)
            acc[i] = d4{0.0, 0.0, 0.0, 0.0};
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int i = 0; i < 8; ++i)
                acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
        }
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < 8; ++i)
            s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
        sink[blockIdx.x * blockDim.x + threadIdx.x] = s;
    } else {
        double acc[8];
#pragma unroll
        for (int i = 0; i < 8; ++i)
            acc[i] = 0.0;
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int i = 0; i < 8; ++i)
                acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[i], 0, 0, 0);
        }
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < 8; ++i)
            s += acc[i];
        sink[blockIdx.x * blockDim.x + threadIdx.x] = s;
    }
}

static void check(hipError_t e, const char *w)
{
    if (e != hipSuccess) {
        fprintf(stderr, "%s: %s\n", w, hipGetErrorString(e));
        exit(1);
    }
}

int main()
{
    double *d, h[64];
    check(hipMalloc(&d, 64 * sizeof(double)), "malloc");
    for (int which = 0; which < 2; ++which) {
        printf("%s operand -> D lanes (v_mfma_f64_4x4x4_16b_f64)\n", which == 0 ? "A" : "B");
        for (int half = 0; half < 2; ++half) {
            hipLaunchKernelGGL(map_kernel, dim3(1), dim3(64), 0, 0, which, half, d);
            check(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost), "copy");
            for (int l = 0; l < 64; ++l) {
                unsigned long long m = (unsigned long long)h[l];
                if (!m)
                    continue;
                printf("  D lane %2d <-", l);
                for (int b = 0; b < 32; ++b)
                    if (m >> b & 1)
                        printf(" %d", b + 32 * half);
                printf("\n");
            }
        }
    }
    double *sink;
    const int blocks = 256 * 16, iters = 2000;
    check(hipMalloc(&sink, (size_t)blocks * 256 * sizeof(double)), "malloc");
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int kind = 0; kind < 2; ++kind) {
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(e0);
            if (kind == 0)
                hipLaunchKernelGGL(rate_kernel<0>, dim3(blocks), dim3(256), 0, 0, sink, iters);
            else
                hipLaunchKernelGGL(rate_kernel<1>, dim3(blocks), dim3(256), 0, 0, sink, iters);
            hipEventRecord(e1);
            check(hipEventSynchronize(e1), "sync");
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            const double insts = (double)blocks * 4 * iters * 8; /* wave instructions */
            printf("%s: %.3f ms, %.3f TFLOP/s (2048 FLOP per wave instruction)\n",
                   kind == 0 ? "16x16x4_f64" : "4x4x4_16b_f64", ms, insts * 2048 / (ms * 1e-3) / 1e12);
        }
    }
    return 0;
}
