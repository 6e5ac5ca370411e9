// HBM read-pattern microbenchmark (measurement tool, not product code):
// how fast 64-70 MB of theory rows can be read on one MI355X with the access
// patterns of the binning / window kernels.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

// 1: fully coalesced grid-stride double2 stream
__global__ void k_stream(const double2 *__restrict__ p, size_t n2, double *out) {
    double s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n2; i += (size_t)gridDim.x * blockDim.x) {
        double2 v = p[i];
        s += v.x + v.y;
    }
    if (s == 1.2345) out[0] = s;
}

// 2: walker rows: W rows of `row` doubles read from a [W][ld] layout; a wave
// covers 16 rows x 64 l (lane: row li, quarter kq, 16 contiguous doubles),
// chunks of 64 l looped `nch` times; grid = (W/64 tiles) x segments
__global__ __launch_bounds__(256) void k_rows(const double *__restrict__ p, long long ld, int row, int nch, int W,
                                              double *out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, li = lane & 15, kq = lane >> 4;
    const int w = blockIdx.x * 64 + wave * 16 + li;
    const int l0 = blockIdx.y * nch * 64;
    const double *r = p + (long long)w * ld;
    double s = 0;
    for (int ch = 0; ch < nch; ch++) {
        const int lb = l0 + ch * 64 + 16 * kq;
        if (lb + 15 < row) {
            const double2 *q = reinterpret_cast<const double2 *>(r + lb);
#pragma unroll
            for (int u = 0; u < 8; u++) { double2 v = q[u]; s += v.x * v.y; }
        }
    }
    if (s == 1.2345) out[0] = s;
}

// 3: walker rows, coalesced along l: a wave reads 64 consecutive double2 of one
// row (1 KB), each block loops rows
__global__ __launch_bounds__(256) void k_rows_lmajor(const double *__restrict__ p, long long ld, int row, int W,
                                                     int rows_per_block, double *out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int seg = blockIdx.y;   // 512 doubles per segment
    double s = 0;
    for (int k = wave; k < rows_per_block; k += 4) {
        const int w = blockIdx.x * rows_per_block + k;
        if (w >= W) break;
        const double2 *q = reinterpret_cast<const double2 *>(p + (long long)w * ld + seg * 512);
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int i = lane + 64 * u;
            if (seg * 512 + 2 * i + 1 < row) { double2 v = q[i]; s += v.x * v.y; }
        }
    }
    if (s == 1.2345) out[0] = s;
}

template <class F> static float timeit(F f, int it = 30) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (int i = 0; i < 3; i++) f();
    CK(hipEventRecord(a));
    for (int i = 0; i < it; i++) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1000.f / it;
}

int main() {
    const int W = 1024;
    const long long ld = 10 * 2560;          // [W][10 fields][2560]: bench-like walker stride
    const int row = 8192;                    // doubles read per walker (~ lensing's 8640)
    const size_t n = (size_t)W * ld;
    double *p, *out;
    CK(hipMalloc(&p, n * 8)); CK(hipMalloc(&out, 8));
    CK(hipMemset(p, 0, n * 8));
    const double mb = (double)W * row * 8 / 1e6;
    // 1: contiguous 64 MB
    size_t n2 = (size_t)W * row / 2;
    for (int blocks : {1024, 2048, 4096, 8192}) {
        float us = timeit([&] { hipLaunchKernelGGL(k_stream, dim3(blocks), dim3(256), 0, 0, (const double2 *)p, n2, out); });
        printf("stream      blocks %5d: %7.2f us  %7.1f GB/s\n", blocks, us, mb * 1e3 / us);
    }
    for (int nch : {1, 2, 4, 8}) {
        dim3 g(W / 64, row / (64 * nch));
        float us = timeit([&] { hipLaunchKernelGGL(k_rows, g, dim3(256), 0, 0, p, ld, row, nch, W, out); });
        printf("rows  nch %d grid %4d: %7.2f us  %7.1f GB/s\n", nch, g.x * g.y, us, mb * 1e3 / us);
        float us2 = timeit([&] { hipLaunchKernelGGL(k_rows, g, dim3(256), 0, 0, p, (long long)row, row, nch, W, out); });
        printf("rows dense nch %d     : %7.2f us  %7.1f GB/s\n", nch, us2, mb * 1e3 / us2);
    }
    for (int rpb : {4, 8, 16, 32}) {
        dim3 g((W + rpb - 1) / rpb, row / 512);
        float us = timeit([&] { hipLaunchKernelGGL(k_rows_lmajor, g, dim3(256), 0, 0, p, ld, row, W, rpb, out); });
        printf("lmajor rpb %2d grid %5d: %7.2f us  %7.1f GB/s\n", rpb, g.x * g.y, us, mb * 1e3 / us);
    }
    return 0;
}
