// Window-kernel anatomy microbenchmark (measurement tool, not product code):
// the read loop of tools/membench2.hip with the window kernel's other parts
// added one at a time -- a per-step workgroup barrier (BAR), the weight tile
// through registers and LDS (WLD), the f64 MFMAs (MF, NB column blocks), the
// XCD-aware item-per-XCD block order (XCD) -- to find what separates the
// kernel (4.5 TB/s with its MFMAs removed) from the bare read (6.2 TB/s).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
typedef double f64x4 __attribute__((ext_vector_type(4)));

template <bool BAR, bool WLD, bool MF, int NB, bool XCD, bool DUAL = false>
__global__ __launch_bounds__(256) void k_win(const double *__restrict__ p, const double *__restrict__ wts, long long ldw,
                                             long long ldf, int seglen, int nseg, int tiles, int nitem, double *out) {
    constexpr int LPL = 8, STEP = 32, WROW = 34;
    __shared__ double wsh[2 * 2 * 16 * WROW];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, li = lane & 15, kq = lane >> 4, tid = threadIdx.x;
    int item, tile;
    if (XCD) {
        const int b = blockIdx.x, xcd = b & 7, j = b >> 3;
        item = xcd + 8 * (j / tiles);
        tile = j % tiles;
        if (item >= nitem) return;
    } else {
        tile = blockIdx.x % tiles;
        item = blockIdx.x / tiles;
    }
    const int field = item / nseg, seg = item % nseg;
    const int w = tile * 64 + wave * 16 + li;
    const double *r = p + (long long)w * ldw + (long long)field * ldf + seg * seglen;
    const int nstep = seglen / STEP;
    double t[LPL], tn[LPL], a[LPL];
    auto load = [&](int st, double *d) {
#pragma unroll
        for (int q = 0; q < LPL / 2; q++) {
            const double2 v = *reinterpret_cast<const double2 *>(r + st * STEP + 8 * q + 2 * kq);
            d[2 * q] = v.x;
            d[2 * q + 1] = v.y;
        }
    };
    const int wc = tid >> 4, wp = 2 * (tid & 15);
    const double *wbase = wts + (long long)item * nstep * 2 * 16 * STEP;
    double2 wr0{}, wr1{};
    auto fetch_w = [&](int st) {
        const double *b0 = wbase + (long long)st * 2 * 16 * STEP + wc * STEP + wp;
        wr0 = *reinterpret_cast<const double2 *>(b0);
        if (NB > 1) wr1 = *reinterpret_cast<const double2 *>(b0 + 16 * STEP);
    };
    auto store_w = [&](int buf) {
        *reinterpret_cast<double2 *>(wsh + ((buf * 2) * 16 + wc) * WROW + wp) = wr0;
        if (NB > 1) *reinterpret_cast<double2 *>(wsh + ((buf * 2 + 1) * 16 + wc) * WROW + wp) = wr1;
    };
    f64x4 acc0 = {0, 0, 0, 0}, acc1 = acc0, bcc0 = acc0, bcc1 = acc0;
    double s = 0;
    load(0, t);
    if (WLD) {
        fetch_w(0);
        store_w(0);
    }
    if (BAR || WLD) __syncthreads();
    for (int st = 0; st < nstep; st++) {
        const bool more = st + 1 < nstep;
        const int cur = st & 1;
        if (more) {
            load(st + 1, tn);
            if (WLD) fetch_w(st + 1);
        }
        if (WLD) {
#pragma unroll
            for (int cb = 0; cb < NB; cb++) {
                const double *src = wsh + ((cur * 2 + cb) * 16 + li) * WROW + 2 * kq;
#pragma unroll
                for (int q = 0; q < LPL / 2; q++) {
                    const double2 v = *reinterpret_cast<const double2 *>(src + 8 * q);
                    a[2 * q] = v.x;
                    a[2 * q + 1] = v.y;
                }
                if (MF && DUAL) {
#pragma unroll
                    for (int u = 0; u < LPL; u += 2) {
                        if (cb == 0) {
                            acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u], t[u], acc0, 0, 0, 0);
                            bcc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u + 1], t[u + 1], bcc0, 0, 0, 0);
                        } else {
                            acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u], t[u], acc1, 0, 0, 0);
                            bcc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u + 1], t[u + 1], bcc1, 0, 0, 0);
                        }
                    }
                } else if (MF) {
#pragma unroll
                    for (int u = 0; u < LPL; u++) {
                        if (cb == 0) acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u], t[u], acc0, 0, 0, 0);
                        else acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u], t[u], acc1, 0, 0, 0);
                    }
                } else {
#pragma unroll
                    for (int u = 0; u < LPL; u++) s += a[u] * t[u];
                }
            }
        } else if (MF) {
#pragma unroll
            for (int u = 0; u < LPL; u++) acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(t[u], t[u], acc0, 0, 0, 0);
        } else {
#pragma unroll
            for (int u = 0; u < LPL; u++) s += t[u] * t[(u + 1) % LPL];
        }
        if (more) {
            if (WLD) store_w(cur ^ 1);
            if (BAR || WLD) __syncthreads();
#pragma unroll
            for (int u = 0; u < LPL; u++) t[u] = tn[u];
        }
    }
    s += acc0[0] + acc0[1] + acc1[2] + acc1[3] + bcc0[0] + bcc1[1];
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

template <bool BAR, bool WLD, bool MF, int NB, bool XCD, bool DUAL = false>
static void run(const double *p, const double *w, double *out, const char *name) {
    const int W = 1024, tiles = W / 64, nfield = 4, seglen = 256, nseg = 2048 / seglen, nitem = nfield * nseg;
    const long long ldf = 2512, ldw = 10 * ldf;
    const double mb = (double)W * nfield * 2048 * 8 / 1e6;
    const int grid = XCD ? 8 * tiles * ((nitem + 7) / 8) : tiles * nitem;
    float us = timeit([&] {
        hipLaunchKernelGGL((k_win<BAR, WLD, MF, NB, XCD, DUAL>), dim3(grid), dim3(256), 0, 0, p, w, ldw, ldf, seglen, nseg,
                           tiles, nitem, out);
    });
    printf("%-34s %7.2f us %7.1f GB/s\n", name, us, mb * 1e3 / us);
}

int main() {
    const size_t n = (size_t)1024 * 10 * 2512 + 4096;
    double *p, *w, *out;
    CK(hipMalloc(&p, n * 8)); CK(hipMalloc(&w, (size_t)32 * 8 * 2 * 16 * 32 * 8)); CK(hipMalloc(&out, 8));
    // non-zero data: a pseudo-random fill
    double *h = (double *)malloc(n * 8);
    for (size_t i = 0; i < n; i++) h[i] = 1.0 + (double)((i * 2654435761u) % 1000) * 1e-3;
    CK(hipMemcpy(p, h, n * 8, hipMemcpyHostToDevice));
    CK(hipMemset(w, 0, (size_t)32 * 8 * 2 * 16 * 32 * 8));
    run<false, false, false, 1, false>(p, w, out, "read");
    run<false, false, false, 1, true>(p, w, out, "read xcd");
    run<true, false, false, 1, true>(p, w, out, "read xcd bar");
    run<true, true, false, 1, true>(p, w, out, "read xcd bar wld");
    run<true, true, false, 2, true>(p, w, out, "read xcd bar wld nb2");
    run<true, true, true, 1, true>(p, w, out, "read xcd bar wld mfma");
    run<true, true, true, 2, true>(p, w, out, "read xcd bar wld mfma nb2");
    run<true, true, true, 1, false>(p, w, out, "read bar wld mfma (linear)");
    run<true, true, true, 1, true, true>(p, w, out, "read xcd bar wld mfma dual");
    run<true, true, true, 2, true, true>(p, w, out, "read xcd bar wld mfma nb2 dual");
    run<false, false, true, 1, true>(p, w, out, "read xcd mfma");
    return 0;
}
