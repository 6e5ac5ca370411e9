// Window-kernel read-pattern microbenchmark (measurement tool, not product
// code): 1024 walker rows [W][10 fields][2512], a field's 2048-l segment read
// by 64-walker workgroups in steps, per-lane granularity LPL doubles per step
// and a prefetch distance of PD steps, as cmbl_window_direct does.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int LPL, int PD, bool INTERLEAVE>
__global__ __launch_bounds__(256) void k_win(const double *__restrict__ p, long long ldw, long long ldf, int seglen,
                                             int nseg, int tiles, double *out) {
    constexpr int STEP = 4 * LPL;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, li = lane & 15, kq = lane >> 4;
    const int tile = blockIdx.x % tiles, item = blockIdx.x / tiles;
    const int field = item / nseg, seg = item % nseg;
    const int w = tile * 64 + wave * 16 + li;
    const double *r = p + (long long)w * ldw + (long long)field * ldf + seg * seglen;
    const int nstep = seglen / STEP;
    double buf[PD + 1][LPL];
    double s = 0;
    auto load = [&](int st, double *d) {
#pragma unroll
        for (int q = 0; q < LPL / 2; q++) {
            const int off = INTERLEAVE ? st * STEP + 8 * q + 2 * kq : st * STEP + LPL * kq + 2 * q;
            const double2 v = *reinterpret_cast<const double2 *>(r + off);
            d[2 * q] = v.x;
            d[2 * q + 1] = v.y;
        }
    };
#pragma unroll
    for (int k = 0; k < PD; k++) load(k, buf[k]);
    for (int st = 0; st < nstep; st++) {
        if (st + PD < nstep) load(st + PD, buf[PD]);
#pragma unroll
        for (int u = 0; u < LPL; u++) s += buf[0][u] * buf[0][(u + 1) % LPL];
#pragma unroll
        for (int k = 0; k < PD; k++)
#pragma unroll
            for (int u = 0; u < LPL; u++) buf[k][u] = buf[k + 1][u];
    }
    if (s == 1.2345) out[0] = s;
}

template <class F> static float timeit(F f, int it = 50) {
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

template <int LPL, int PD, bool IL>
static void run(const double *p, double *out, int seglen) {
    const int W = 1024, tiles = W / 64, nfield = 4, nseg = 2048 / seglen;
    const long long ldf = 2512, ldw = 10 * ldf;
    const double mb = (double)W * nfield * 2048 * 8 / 1e6;
    float us = timeit([&] {
        hipLaunchKernelGGL((k_win<LPL, PD, IL>), dim3(tiles * nfield * nseg), dim3(256), 0, 0, p, ldw, ldf, seglen,
                           nseg, tiles, out);
    });
    printf("LPL %2d PD %d %s seg %4d grid %4d: %7.2f us %7.1f GB/s\n", LPL, PD, IL ? "interleaved" : "blocked    ",
           seglen, tiles * nfield * nseg, us, mb * 1e3 / us);
}

int main() {
    const size_t n = (size_t)1024 * 10 * 2512 + 4096;
    double *p, *out;
    CK(hipMalloc(&p, n * 8)); CK(hipMalloc(&out, 8));
    CK(hipMemset(p, 0, n * 8));
    for (int seg : {256, 512, 128}) {
        run<8, 1, true>(p, out, seg);
        run<8, 2, true>(p, out, seg);
        run<8, 3, true>(p, out, seg);
        run<8, 1, false>(p, out, seg);
        run<16, 1, false>(p, out, seg);
        run<16, 2, false>(p, out, seg);
        run<4, 2, true>(p, out, seg);
        run<4, 4, true>(p, out, seg);
    }
    return 0;
}
