// f64 MFMA throughput microbenchmark (measurement tool): v_mfma_f64_16x16x4f64
// with NACC independent accumulators, operands in registers.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double f64x4 __attribute__((ext_vector_type(4)));
template <int NACC>
__global__ __launch_bounds__(256) void k(double *out, int iters, double a0, double b0) {
    f64x4 acc[NACC];
    for (int i = 0; i < NACC; i++) acc[i] = f64x4{0, 0, 0, 0};
    double a = a0 + threadIdx.x, b = b0 - threadIdx.x;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < NACC; i++) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    }
    double s = 0;
    for (int i = 0; i < NACC; i++) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    if (s == 1.2345) out[0] = s;
}
template <int NACC> void run(int blocks_per_cu, double *out) {
    const int iters = 4096, blocks = 256 * blocks_per_cu;
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(k<NACC>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0, 2.0);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<NACC>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0, 2.0);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double flops = (double)blocks * 4 * iters * NACC * 2.0 * 16 * 16 * 4;
    printf("NACC %d waves/SIMD %d: %.2f ms  %.1f TF\n", NACC, blocks_per_cu, ms, flops / ms / 1e9);
}
int main() {
    double *out; hipMalloc(&out, 8);
    for (int b : {1, 2, 4}) { run<1>(b, out); run<2>(b, out); run<4>(b, out); run<8>(b, out); }
    return 0;
}
