// Microbenchmark: f64 MFMA (v_mfma_f64_16x16x4f64) throughput on gfx950.
// Each wave runs NACC independent accumulator chains of ITERS MFMAs.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double f64x4 __attribute__((ext_vector_type(4)));
template <int NACC>
__global__ __launch_bounds__(256) void k(double *out, int iters, double a0, double b0) {
    f64x4 acc[NACC];
    for (int i = 0; i < NACC; i++) acc[i] = f64x4{0, 0, 0, 0};
    double a = a0 + threadIdx.x * 1e-9, b = b0 - threadIdx.x * 1e-9;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < NACC; i++) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    }
    double s = 0;
    for (int i = 0; i < NACC; i++) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
int main() {
    int ncu = 256;
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    ncu = p.multiProcessorCount;
    double *out;
    hipMalloc(&out, sizeof(double) * ncu * 8 * 256);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 4000;
    for (int rep = 0; rep < 2; rep++) {
        for (int blocksPerCU : {1, 2}) {
            int blocks = ncu * blocksPerCU;
            hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(256), 0, 0, out, 10, 1.0, 1.0);
            hipEventRecord(e0);
            hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0, 1.0);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            double flops = 2.0 * 16 * 16 * 4 * 4.0 * iters * (blocks * 4);
            printf("NACC=4 blocks/CU=%d: %.3f ms  %.1f TFLOP/s  (%.1f cycles/MFMA/SIMD at 2.4GHz, 1 wave/SIMD per block)\n",
                   blocksPerCU, ms, flops / ms / 1e9, ms * 1e-3 * 2.4e9 / (iters * 4.0 * blocksPerCU));
        }
        int blocks = ncu;
        hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, 10, 1.0, 1.0);
        hipEventRecord(e0);
        hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0, 1.0);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("NACC=1 (dependent chain): %.3f ms -> %.1f cycles latency per MFMA at 2.4GHz\n", ms,
               ms * 1e-3 * 2.4e9 / iters);
    }
    printf("CUs=%d clock(kHz)=%d\n", ncu, p.clockRate);
    return 0;
}
