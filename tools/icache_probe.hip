// Instruction-fetch cost probe: one wave runs the same straight-line block
// of 4-byte VALU instructions twice (cold, then warm in the instruction
// cache) and stamps each pass with s_memtime.  Grids of 1 / 64 / 256
// workgroups, optionally beside a streaming kernel on another stream.
//   hipcc -O3 --offload-arch=gfx950 tools/icache_probe.hip -o tools/_icache_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define BLOCK_ASM(N)                                                                          \
    asm volatile(".rept " #N "\n v_add_u32 %0, 1, %0\n v_add_u32 %1, 1, %1\n .endr"          \
                 : "+v"(a), "+v"(b))

template <int KB>
__global__ __launch_bounds__(64) void probe(unsigned long long *out)
{
    unsigned a = threadIdx.x, b = 2 * threadIdx.x;
    unsigned long long t[3];
    for (int it = 0; it < 2; it++) {
        t[it] = __builtin_amdgcn_s_memtime();
        if constexpr (KB == 4) BLOCK_ASM(512);
        if constexpr (KB == 16) BLOCK_ASM(2048);
        if constexpr (KB == 48) BLOCK_ASM(6144);
    }
    t[2] = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
        out[3 * blockIdx.x + 0] = t[1] - t[0];
        out[3 * blockIdx.x + 1] = t[2] - t[1];
        out[3 * blockIdx.x + 2] = a + b;
    }
}

__global__ void stream_kernel(const double4 *src, double *dst, size_t n, int reps)
{
    double s = 0;
    for (int r = 0; r < reps; r++)
        for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
            const double4 v = src[i];
            s += v.x + v.y + v.z + v.w;
        }
    if (s == 12345.0) dst[0] = s;
}

template <int KB>
static void run(int grid, bool streaming, hipStream_t s1, hipStream_t s2, const double4 *src, double *dst, size_t n)
{
    unsigned long long *d;
    hipMalloc(&d, 3 * 8 * grid);
    if (streaming) hipLaunchKernelGGL(stream_kernel, dim3(2048), dim3(256), 0, s2, src, dst, n, 4);
    hipLaunchKernelGGL(probe<KB>, dim3(grid), dim3(64), 0, s1, d);
    hipDeviceSynchronize();
    std::vector<unsigned long long> h(3 * grid);
    hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
    std::vector<unsigned long long> c0, c1;
    for (int i = 0; i < grid; i++) { c0.push_back(h[3 * i]); c1.push_back(h[3 * i + 1]); }
    std::sort(c0.begin(), c0.end());
    std::sort(c1.begin(), c1.end());
    printf("%2d KB code, grid %4d%s: cold median %7llu max %7llu | warm median %7llu  (s_memtime ticks)\n", KB,
           grid, streaming ? " + streaming" : "            ", c0[grid / 2], c0.back(), c1[grid / 2]);
    hipFree(d);
}

int main()
{
    hipStream_t s1, s2;
    hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
    hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
    const size_t n = (size_t)1 << 25;   // 1 GiB of double4
    double4 *src;
    double *dst;
    hipMalloc(&src, n * sizeof(double4));
    hipMemset(src, 0, n * sizeof(double4));
    hipMalloc(&dst, 64);
    for (int rep = 0; rep < 2; rep++) {
        for (int g : {1, 64, 256}) {
            run<4>(g, false, s1, s2, src, dst, n);
            run<16>(g, false, s1, s2, src, dst, n);
            run<48>(g, false, s1, s2, src, dst, n);
        }
        for (int g : {64}) {
            run<16>(g, true, s1, s2, src, dst, n);
            run<48>(g, true, s1, s2, src, dst, n);
        }
    }
    hipFree(src);
    hipFree(dst);
    return 0;
}
