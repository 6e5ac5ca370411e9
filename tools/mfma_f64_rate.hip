// f64 MFMA ceiling on gfx950: v_mfma_f64_16x16x4_f64 issued from inline asm
// so the accumulators stay in VGPRs (the compiled-intrinsic probe,
// mfma_f64_probe.hip, round-trips them through AGPRs every iteration and
// under-reads the pipe).  Reports, per configuration, TFLOP/s over the
// launch (HIP events), the in-kernel clock (s_memtime vs s_memrealtime) and
// cycles per MFMA per SIMD.
//   chain  : one wave per SIMD, NACC independent accumulators round-robin
//   waves  : W waves per SIMD (blocks of 256 = 4 waves, one per SIMD)
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double f64x4 __attribute__((ext_vector_type(4)));

#define MFMA(acc, a, b) asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b))

template <int NACC>
__global__ __launch_bounds__(256) void kmfma(double *out, unsigned long long *clk, int iters, double a0, double b0)
{
    f64x4 acc[NACC];
#pragma unroll
    for (int i = 0; i < NACC; i++) acc[i] = f64x4{0, 0, 0, 0};
    const double a = a0 + threadIdx.x * 1e-9, b = b0 - threadIdx.x * 1e-9;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < NACC; i++) MFMA(acc[i], a, b);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    double s = 0;
#pragma unroll
    for (int i = 0; i < NACC; i++) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
}

template <class K>
static void run(const char *name, K kern, int blocks, int iters, int nacc, double *out, unsigned long long *clk)
{
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, clk, 50, 1.0, 1.0);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, clk, iters, 1.0, 1.0);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long c[2];
    (void)hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
    const double ghz = (double)c[0] / ((double)c[1] / 100e6) / 1e9;     // s_memrealtime: 100 MHz
    const double mfmas = (double)iters * nacc * blocks * 4;             // wave-level MFMAs (4 waves/block)
    const double tf = mfmas * 2048.0 / (ms * 1e-3) / 1e12;              // 16x16x4: 2048 flop per wave MFMA
    const double waves_per_simd = blocks * 4.0 / 1024.0;
    const double cyc_per_mfma = (double)c[0] / (iters * nacc * waves_per_simd);   // per SIMD, block 0's window
    printf("%-10s nacc=%2d blocks=%5d waves/SIMD=%4.1f  %8.3f ms  %6.1f TFLOP/s  clock %.2f GHz  %.1f cyc/MFMA/SIMD\n",
           name, nacc, blocks, waves_per_simd, ms, tf, ghz, cyc_per_mfma);
}

int main()
{
    double *out;
    unsigned long long *clk;
    (void)hipMalloc(&out, sizeof(double) * 256 * 4096);
    (void)hipMalloc(&clk, 16);
    const int it = 4000;
    run("latency", kmfma<1>, 256, it, 1, out, clk);      // one dependent chain per wave, one wave per SIMD
    run("chain", kmfma<2>, 256, it, 2, out, clk);
    run("chain", kmfma<4>, 256, it, 4, out, clk);
    run("chain", kmfma<8>, 256, it, 8, out, clk);
    for (int bpc : {2, 4}) {
        run("waves", kmfma<4>, 256 * bpc, it, 4, out, clk);
        run("waves", kmfma<8>, 256 * bpc, it, 8, out, clk);
    }
    return 0;
}
