// Microbenchmark: f64 MFMA (v_mfma_f64_16x16x4f64) and f64 VALU FMA
// throughput on gfx950, with the in-kernel clock (s_memtime / s_memrealtime).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double f64x4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void kmfma(double *out, unsigned long long *clk, int iters, double a0, double b0) {
    f64x4 acc[NACC];
    for (int i = 0; i < NACC; i++) acc[i] = f64x4{0, 0, 0, 0};
    double a = a0 + threadIdx.x * 1e-9, b = b0 - threadIdx.x * 1e-9;
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < NACC; i++) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    double s = 0;
    for (int i = 0; i < NACC; i++) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

template <int NACC>
__global__ __launch_bounds__(256) void kvalu(double *out, unsigned long long *clk, int iters, double a0, double b0) {
    double acc[NACC];
    for (int i = 0; i < NACC; i++) acc[i] = i * 1e-3;
    double a = a0 + threadIdx.x * 1e-9, b = b0 - threadIdx.x * 1e-9;
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < NACC; i++) acc[i] = __builtin_fma(a, acc[i], b);
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    double s = 0;
    for (int i = 0; i < NACC; i++) s += acc[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

template <class K>
void run(const char *name, K kern, int blocks, int iters, double flops_per_thread_iter, double *out,
         unsigned long long *clk) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, clk, 20, 1.0, 1.0);
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, clk, iters, 1.0, 1.0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long c[2];
    hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
    const double ghz = (double)c[0] / ((double)c[1] / 100e6) / 1e9;   // s_memrealtime = 100 MHz
    const double tf = flops_per_thread_iter * iters * blocks * 256.0 / (ms * 1e-3) / 1e12;
    printf("%-28s blocks=%5d  %.3f ms  %6.1f TFLOP/s  clock %.2f GHz\n", name, blocks, ms, tf, ghz);
}

int main() {
    double *out;
    unsigned long long *clk;
    hipMalloc(&out, sizeof(double) * 256 * 8 * 256);
    hipMalloc(&clk, 16);
    const int it = 3000;
    // f64 16x16x4 MFMA: 2*16*16*4 = 2048 flop per wave per MFMA = 32 per lane
    for (int bpc : {1, 2, 4}) {
        run("mfma NACC=4", kmfma<4>, 256 * bpc, it, 32.0 * 4, out, clk);
        run("mfma NACC=8", kmfma<8>, 256 * bpc, it, 32.0 * 8, out, clk);
        run("mfma NACC=16", kmfma<16>, 256 * bpc, it / 2, 32.0 * 16, out, clk);
    }
    for (int bpc : {1, 2, 4, 8}) {
        run("valu fma NACC=8", kvalu<8>, 256 * bpc, it * 4, 2.0 * 8, out, clk);
        run("valu fma NACC=16", kvalu<16>, 256 * bpc, it * 2, 2.0 * 16, out, clk);
    }
    return 0;
}
