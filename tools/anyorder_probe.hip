// Probe: do two independent kernels on ONE stream overlap when the second is
// launched with hipExtAnyOrderLaunch (AQL barrier bit clear)?  Three proxies of
// the sampler step's kernels: S streams ~80 MB of HBM (the fused window pass),
// M runs f64 MFMA chains on every CU (the quadform), L is a 16-workgroup
// dependent latency chain (mh_kernel).  Prints the time of each alone and of
// pairs launched in order vs any-order.
//   hipcc -O3 --offload-arch=gfx950 tools/anyorder_probe.hip -o tools/_anyorder && ./tools/_anyorder
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
            return 1;                                                                     \
        }                                                                                 \
    } while (0)

typedef double f64x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void stream_k(const double2 *__restrict__ src, long long n2, double *out)
{
    double2 acc{0.0, 0.0};
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n2; i += (long long)gridDim.x * 256) {
        const double2 v = src[i];
        acc.x += v.x;
        acc.y += v.y;
    }
    if (acc.x == 12345.678) out[0] = acc.y;
}

__global__ __launch_bounds__(256) void mfma_k(int iters, double *out)
{
    f64x4 a0 = {0, 0, 0, 0}, a1 = a0, a2 = a0, a3 = a0;
    double x = threadIdx.x * 1e-3, y = blockIdx.x * 1e-3;
    for (int i = 0; i < iters; i++) {
        a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(y, x, a1, 0, 0, 0);
        a2 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x, a2, 0, 0, 0);
        a3 = __builtin_amdgcn_mfma_f64_16x16x4f64(y, y, a3, 0, 0, 0);
    }
    const double s = a0[0] + a1[1] + a2[2] + a3[3];
    if (s == 12345.678) out[1] = s;
}

__global__ __launch_bounds__(64) void chain_k(int iters, double *out)
{
    __shared__ double u[97 * 64];
    for (int i = 0; i < 97; i++) u[i * 64 + threadIdx.x] = (i + 1) * 0.0103;
    double c = 0.3;
    int i97 = 97, j97 = 33;
    for (int k = 0; k < iters; k++) {   // a RANMAR-like dependent chain through LDS
        double uni = u[(i97 - 1) * 64 + threadIdx.x] - u[(j97 - 1) * 64 + threadIdx.x];
        if (uni < 0) uni += 1.0;
        u[(i97 - 1) * 64 + threadIdx.x] = uni;
        if (--i97 == 0) i97 = 97;
        if (--j97 == 0) j97 = 97;
        c = c - 0.456;
        if (c < 0) c += 0.99;
        c = log(c + uni + 1.0);
    }
    if (c == 12345.678) out[2] = c;
}

int main()
{
    const long long bytes = 80ll << 20, n2 = bytes / 16;
    double2 *src;
    double *out;
    CK(hipMalloc(&src, bytes));
    CK(hipMemset(src, 0, bytes));
    CK(hipMalloc(&out, 64));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int mfma_iters = 36, chain_iters = 45;
    auto S = [&](unsigned fl) {
        hipExtLaunchKernelGGL(stream_k, dim3(2048), dim3(256), 0, st, nullptr, nullptr, fl, (const double2 *)src, n2, out);
    };
    auto M = [&](unsigned fl) { hipExtLaunchKernelGGL(mfma_k, dim3(512), dim3(256), 0, st, nullptr, nullptr, fl, mfma_iters, out); };
    auto L = [&](unsigned fl) { hipExtLaunchKernelGGL(chain_k, dim3(16), dim3(64), 0, st, nullptr, nullptr, fl, chain_iters, out); };
    auto timeit = [&](const char *name, auto body) {
        for (int w = 0; w < 5; w++) body();
        CK(hipStreamSynchronize(st));
        const int reps = 50;
        CK(hipEventRecord(e0, st));
        for (int r = 0; r < reps; r++) body();
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-34s %8.2f us\n", name, ms * 1e3 / reps);
        return 0;
    };
    timeit("S (80 MB stream)", [&] { S(0); });
    timeit("M (mfma, 512 wg)", [&] { M(0); });
    timeit("L (16-wg latency chain)", [&] { L(0); });
    timeit("S;M in order", [&] { S(0); M(0); });
    timeit("S;M any-order", [&] { S(0); M(hipExtAnyOrderLaunch); });
    timeit("S;L in order", [&] { S(0); L(0); });
    timeit("S;L any-order", [&] { S(0); L(hipExtAnyOrderLaunch); });
    timeit("L;S any-order", [&] { L(0); S(hipExtAnyOrderLaunch); });
    timeit("M;L in order", [&] { M(0); L(0); });
    timeit("M;L any-order", [&] { M(0); L(hipExtAnyOrderLaunch); });
    timeit("S;M;L in order", [&] { S(0); M(0); L(0); });
    timeit("S;L(ao) M;L(ao)", [&] { S(0); L(hipExtAnyOrderLaunch); M(0); L(hipExtAnyOrderLaunch); });
    // two independent walker groups, each a chain L -> S/2 -> M/2 per step, on
    // one stream (serial) or on two streams (no per-step events)
    hipStream_t s2;
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    auto Sh = [&](hipStream_t q) {
        hipExtLaunchKernelGGL(stream_k, dim3(1024), dim3(256), 0, q, nullptr, nullptr, 0, (const double2 *)src, n2 / 2, out);
    };
    auto Mh = [&](hipStream_t q) { hipExtLaunchKernelGGL(mfma_k, dim3(256), dim3(256), 0, q, nullptr, nullptr, 0, mfma_iters, out); };
    auto Lq = [&](hipStream_t q) { hipExtLaunchKernelGGL(chain_k, dim3(8), dim3(64), 0, q, nullptr, nullptr, 0, chain_iters, out); };
    auto Sf = [&](hipStream_t q) {
        hipExtLaunchKernelGGL(stream_k, dim3(2048), dim3(256), 0, q, nullptr, nullptr, 0, (const double2 *)src, n2, out);
    };
    auto Mf = [&](hipStream_t q) { hipExtLaunchKernelGGL(mfma_k, dim3(512), dim3(256), 0, q, nullptr, nullptr, 0, mfma_iters, out); };
    auto Lf = [&](hipStream_t q) { hipExtLaunchKernelGGL(chain_k, dim3(16), dim3(64), 0, q, nullptr, nullptr, 0, chain_iters, out); };
    timeit("full W: L;S;M one stream", [&] { Lf(st); Sf(st); Mf(st); });
    timeit("2 groups one stream", [&] { Lq(st); Sh(st); Mh(st); Lq(st); Sh(st); Mh(st); });
    auto two = [&](const char *name, int reps) {
        for (int w = 0; w < 3; w++) { Lq(st); Sh(st); Mh(st); Lq(s2); Sh(s2); Mh(s2); }
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, st));
        CK(hipStreamWaitEvent(s2, e0, 0));
        for (int r = 0; r < reps; r++) {
            Lq(st); Sh(st); Mh(st);
            Lq(s2); Sh(s2); Mh(s2);
        }
        hipEvent_t j;
        CK(hipEventCreate(&j));
        CK(hipEventRecord(j, s2));
        CK(hipStreamWaitEvent(st, j, 0));
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-34s %8.2f us\n", name, ms * 1e3 / reps);
        return 0;
    };
    two("2 groups two streams", 50);
    return 0;
}
