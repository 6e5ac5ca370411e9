// Sample collector on device: every walker's TMpiChainCollector Samples list
// (source/SampleCollector.f90:324-460) -- the thinned list of points the
// convergence test and proposal learning window over -- as a per-walker ring
// of history step numbers, plus its burn-in state.
//
//   samp  [samp_cap][ld] int  history step of each stored sample (ring per walker)
//   start, count [ld]         the walker's list = ring slots start .. start+count-1
//   snum, thin [ld]           sample_num and MPI_thin_fac (AddNewPoint :347-348)
//   burn [ld], pchg [n][ld]   Burn_done and param_changes (:352-377)
//
// The points themselves stay in the sampler's history ring (one row per step,
// sampler.hip), so adding a sample is an int write and the window statistics
// gather their rows from it.  Every kernel here is one lane per walker with
// walker-minor (coalesced) state rows.
#include <algorithm>
#include <cmath>
#include <cstring>

#include "sampler.h"

namespace cmamd {

static constexpr double CLOGZERO = CMBL_LOGZERO;

// AddNewPoint for the history steps `steps` (in order) of every walker:
// sample_num++; keep every thin-th; Samples%Add; before burn-in, count
// parameter changes between consecutive samples once Count > 51 and declare
// the burn done when every used parameter changed more than 51 times
// (:352-377), then keep the last min_update samples (DeleteRange, :391-397).
// Points at logZero are never added (SampleFrom, MCMC.f90:146).
__global__ void collector_add_kernel(const double *hist, int hist_cap, int W, int n, const int *steps, int nsteps,
                                     int *samp, int samp_cap, int *start, int *count, int *snum, const int *thin,
                                     int *burn, int *pchg, int min_update, int check_burn, int *overflow)
{
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= W) return;
    int st = start[w], cnt = count[w], sn = snum[w], bd = burn[w];
    const int th = thin[w];
    for (int k = 0; k < nsteps; k++) {
        const int t = steps[k];
        const double *row = hist + (size_t)(t % hist_cap) * (n + 1) * W + w;
        if (row[(size_t)n * W] == CLOGZERO) continue;
        sn++;                                                    // this%sample_num + 1 (:346)
        if (sn % th != 0) continue;                              // MPI_thin_fac (:347)
        if (cnt == samp_cap) {                                   // the ring is full: the caller's capacity is too small
            atomicOr(overflow, 1);
            continue;
        }
        samp[(size_t)((st + cnt) % samp_cap) * W + w] = t;
        cnt++;
        if (!check_burn || bd || cnt <= 51) continue;
        const int prev = samp[(size_t)((st + cnt - 2) % samp_cap) * W + w];
        const double *prow = hist + (size_t)(prev % hist_cap) * (n + 1) * W + w;
        bool all = true;
        for (int i = 0; i < n; i++) {
            int c = pchg[(size_t)i * W + w];
            if (row[(size_t)i * W] != prow[(size_t)i * W]) pchg[(size_t)i * W + w] = ++c;
            all = all && c > 51;
        }
        if (all) {                                               // Burn_done (:371)
            bd = 1;
            if (cnt > min_update) {                              // DeleteRange(1, Count - Min) (:397)
                st = (st + cnt - min_update) % samp_cap;
                cnt = min_update;
            }
            for (int i = 0; i < n; i++) pchg[(size_t)i * W + w] = 0;
        }
    }
    start[w] = st;
    count[w] = cnt;
    snum[w] = sn;
    burn[w] = bd;
}

// Samples%Thin(2) for walkers whose count exceeds `limit` (SampleCollector.f90:300-304;
// TObjectList%Thin, ObjectLists.f90:508-530: items 1, 3, 5, ...), and their
// MPI_thin_fac doubles.  In place: slot k takes slot 2k (2k >= k).
__global__ void collector_thin_kernel(int W, int *samp, int samp_cap, const int *start, int *count, int *thin,
                                      int limit)
{
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= W) return;
    const int cnt = count[w];
    if (cnt <= limit || cnt <= 1) return;
    const int st = start[w];
    const int nc = (cnt - 1) / 2 + 1;
    for (int k = 1; k < nc; k++)
        samp[(size_t)((st + k) % samp_cap) * W + w] = samp[(size_t)((st + 2 * k) % samp_cap) * W + w];
    count[w] = nc;
    thin[w] *= 2;
}

// Per-walker mean and covariance over the second half of its Samples list,
// items Count/2 .. Count (1-based, inclusive; Count - Count/2 + 1 of them),
// two passes as the reference (:233-246).  One block = 64 walkers x HS_PH
// item phases, fixed-order combination (deterministic); the covariance pass
// runs one block per (walker tile, row i).
static constexpr int CPH = 4;

template <int NC>
__global__ __launch_bounds__(64 * CPH) void coll_mean_kernel(const double *hist, int hist_cap, int W, int n,
                                                            const int *samp, int samp_cap, const int *start,
                                                            const int *count, double *means, int *wcount)
{
    __shared__ double part[CPH][NC][64];
    const int lane = threadIdx.x & 63, ph = threadIdx.x >> 6;
    const int w = blockIdx.x * 64 + lane;
    double acc[NC];
#pragma unroll
    for (int j = 0; j < NC; j++) acc[j] = 0.0;
    int c0 = 0;
    if (w < W) {
        const int st = start[w], cnt = count[w];
        const int k0 = cnt / 2 - 1;                              // 0-based item of Count/2
        c0 = cnt - cnt / 2 + 1;
        for (int k = k0 + ph; k < cnt; k += CPH) {
            const int t = samp[(size_t)((st + k) % samp_cap) * W + w];
            const double *row = hist + (size_t)(t % hist_cap) * (n + 1) * W + w;
#pragma unroll
            for (int j = 0; j < NC; j++)
                if (j < n) acc[j] += row[(size_t)j * W];
        }
    }
#pragma unroll
    for (int j = 0; j < NC; j++) part[ph][j][lane] = acc[j];
    __syncthreads();
    if (ph == 0 && w < W) {
        for (int j = 0; j < n; j++) {
            double v = part[0][j][lane];
            for (int p = 1; p < CPH; p++) v += part[p][j][lane];
            means[(size_t)w * n + j] = v / c0;                   // MPIMean / MPImean(0)
        }
        wcount[w] = c0;
    }
}

template <int NC>
__global__ __launch_bounds__(64 * CPH) void coll_cov_kernel(const double *hist, int hist_cap, int W, int n,
                                                           const int *samp, int samp_cap, const int *start,
                                                           const int *count, const double *means, double *covs)
{
    __shared__ double part[CPH][NC][64];
    const int lane = threadIdx.x & 63, ph = threadIdx.x >> 6;
    const int w = blockIdx.x * 64 + lane, i = blockIdx.y;
    double acc[NC], m[NC];
#pragma unroll
    for (int j = 0; j < NC; j++) {
        acc[j] = 0.0;
        m[j] = (w < W && j < n) ? means[(size_t)w * n + j] : 0.0;
    }
    double mi = 0.0;
#pragma unroll
    for (int j = 0; j < NC; j++)
        if (j == i) mi = m[j];
    int c0 = 1;
    if (w < W) {
        const int st = start[w], cnt = count[w];
        c0 = cnt - cnt / 2 + 1;
        for (int k = cnt / 2 - 1 + ph; k < cnt; k += CPH) {
            const int t = samp[(size_t)((st + k) % samp_cap) * W + w];
            const double *row = hist + (size_t)(t % hist_cap) * (n + 1) * W + w;
            const double di = row[(size_t)i * W] - mi;
#pragma unroll
            for (int j = 0; j < NC; j++)
                if (j < n) acc[j] += (row[(size_t)j * W] - m[j]) * di;
        }
    }
#pragma unroll
    for (int j = 0; j < NC; j++) part[ph][j][lane] = acc[j];
    __syncthreads();
    if (ph == 0 && w < W) {
        for (int j = 0; j < n; j++) {
            double v = part[0][j][lane];
            for (int p = 1; p < CPH; p++) v += part[p][j][lane];
            covs[(size_t)w * n * n + (size_t)i * n + j] = v / c0;
        }
    }
}

// ConfidVal (samples.f90:70-110) of every (walker, checked parameter) over the
// walker's window, without sorting: the order statistics at 0-based ranks
// b-1 and b of pos = (samps-1)*limfrac + 1 (and of 1 - limfrac) by a radix
// select on the order-preserving 64-bit keys of the doubles, 8 passes of 8
// bits, 256-bin LDS histogram per pass.  One block of 256 threads per
// (walker, parameter); the window values are gathered from the history ring
// on every pass (the windows are read-mostly L2 traffic at the check cadence).
__device__ inline unsigned long long dkey(double x)
{
    unsigned long long u = __double_as_longlong(x);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__device__ inline double dval(unsigned long long k)
{
    const unsigned long long u = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
    return __longlong_as_double(u);
}

__device__ double select_rank(const double *hist, int hist_cap, int W, int n, const int *samp, int samp_cap, int w,
                              int st, int k0, int cnt, int param, int rank, unsigned *hbin, int *shared_sel)
{
    unsigned long long prefix = 0;
    int r = rank;
    for (int pass = 7; pass >= 0; pass--) {
        const int shift = pass * 8;
        for (int b = threadIdx.x; b < 256; b += blockDim.x) hbin[b] = 0;
        __syncthreads();
        const unsigned long long hi_mask = pass == 7 ? 0ull : (~0ull << (shift + 8));
        for (int k = k0 + threadIdx.x; k < cnt; k += blockDim.x) {
            const int t = samp[(size_t)((st + k) % samp_cap) * W + w];
            const unsigned long long key = dkey(hist[((size_t)(t % hist_cap) * (n + 1) + param) * W + w]);
            if ((key & hi_mask) == prefix) atomicAdd(&hbin[(key >> shift) & 255u], 1u);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            int b = 0;
            while (b < 255 && r >= (int)hbin[b]) {
                r -= (int)hbin[b];
                b++;
            }
            shared_sel[0] = b;
            shared_sel[1] = r;
        }
        __syncthreads();
        prefix |= (unsigned long long)shared_sel[0] << shift;
        r = shared_sel[1];
        __syncthreads();
    }
    return dval(prefix);
}

__global__ __launch_bounds__(256) void coll_limits_kernel(const double *hist, int hist_cap, int W, int n,
                                                          const int *samp, int samp_cap, const int *start,
                                                          const int *count, const int *params, int ncheck,
                                                          double limfrac, double *out)
{
    __shared__ unsigned hbin[256];
    __shared__ int sel[2];
    const int w = blockIdx.x, c = blockIdx.y;
    const int param = params[c];
    const int st = start[w], cnt = count[w];
    const int k0 = cnt / 2 - 1;                                  // ConfidVal(ix, limfrac, Count/2, Count)
    const int samps = cnt - k0;
    double res[2];
    for (int side = 0; side < 2; side++) {
        const double pos = (samps - 1) * (side == 0 ? limfrac : (1.0 - limfrac)) + 1;
        const int b = max((int)pos, 1);
        double v = select_rank(hist, hist_cap, W, n, samp, samp_cap, w, st, k0, cnt, param, b - 1, hbin, sel);
        if (b < samps && pos > b) {
            const double d = pos - b;
            const double v1 = select_rank(hist, hist_cap, W, n, samp, samp_cap, w, st, k0, cnt, param, b, hbin, sel);
            v = v * (1 - d) + d * v1;
        }
        res[side] = v;
    }
    if (threadIdx.x == 0) {
        out[((size_t)w * ncheck + c) * 2] = res[0];
        out[((size_t)w * ncheck + c) * 2 + 1] = res[1];
    }
}

// ------------------------------------------------------------------ host

void sampler_collector_enable(cmbs *s, int samp_capacity) {
    if (s->hist_cap == 0) fail(CMBL_ERR_ARG, "the collector windows over the history ring: cmbs_enable_history first");
    if (samp_capacity <= 0) fail(CMBL_ERR_ARG, "sample capacity must be positive");
    const size_t ld = s->W;
    auto &c = s->coll;
    // already enabled at this capacity: keep the lists (a collector built after
    // cmbs_load_state must not wipe the restored ones)
    if (c.enabled && c.cap == samp_capacity) return;
    c.cap = samp_capacity;
    c.samp.alloc((size_t)samp_capacity * ld * 4);
    c.state.alloc((size_t)(5 + s->n_used) * ld * 4);     // start, count, snum, thin, burn, pchg[n]
    std::vector<int> init((size_t)(5 + s->n_used) * ld, 0);
    for (size_t w = 0; w < ld; w++) init[3 * ld + w] = 1;   // MPI_thin_fac = 1
    c.state.upload(init.data(), init.size() * 4);
    c.flag.alloc(64);
    c.wcount.alloc(ld * 4);
    c.enabled = true;
}

static int *cstate(cmbs *s, int row) { return s->coll.state.as<int>() + (size_t)row * s->W; }

void sampler_collector_add(cmbs *s, const int *steps, int nsteps, int min_update, int check_burn, hipStream_t st) {
    auto &c = s->coll;
    if (!c.enabled) fail(CMBL_ERR_ARG, "collector not enabled");
    if (nsteps <= 0) return;
    for (int k = 0; k < nsteps; k++) {
        if (steps[k] < 0 || steps[k] >= s->hist_count || s->hist_count - steps[k] > s->hist_cap)
            fail(CMBL_ERR_ARG, "history step %d is not in the ring (count %d, capacity %d)", steps[k],
                 s->hist_count, s->hist_cap);
        if (k && steps[k] <= steps[k - 1]) fail(CMBL_ERR_ARG, "collector steps must increase");
    }
    c.steps.grow((size_t)nsteps * 4);
    HIP_CHECK(hipMemcpyAsync(c.steps.p, steps, (size_t)nsteps * 4, hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemsetAsync(c.flag.p, 0, 4, st));
    hipLaunchKernelGGL(collector_add_kernel, dim3((s->W + 63) / 64), dim3(64), 0, st, s->hist.as<double>(),
                       s->hist_cap, s->W, s->n_used, c.steps.as<int>(), nsteps, c.samp.as<int>(), c.cap,
                       cstate(s, 0), cstate(s, 1), cstate(s, 2), cstate(s, 3), cstate(s, 4), cstate(s, 5),
                       min_update, check_burn, c.flag.as<int>());
    HIP_CHECK(hipGetLastError());
    int ovf = 0;
    HIP_CHECK(hipMemcpyAsync(&ovf, c.flag.p, 4, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    if (ovf) fail(CMBL_ERR_ARG, "sample list capacity %d exceeded: enable the collector with a larger capacity", c.cap);
}

void sampler_collector_state_host(cmbs *s, int *start, int *count, int *burn, int *thin) {
    auto &c = s->coll;
    if (!c.enabled) fail(CMBL_ERR_ARG, "collector not enabled");
    HIP_CHECK(hipDeviceSynchronize());
    const size_t b = (size_t)s->W * 4;
    if (start) HIP_CHECK(hipMemcpy(start, cstate(s, 0), b, hipMemcpyDeviceToHost));
    if (count) HIP_CHECK(hipMemcpy(count, cstate(s, 1), b, hipMemcpyDeviceToHost));
    if (thin) HIP_CHECK(hipMemcpy(thin, cstate(s, 3), b, hipMemcpyDeviceToHost));
    if (burn) HIP_CHECK(hipMemcpy(burn, cstate(s, 4), b, hipMemcpyDeviceToHost));
}

void sampler_collector_thin(cmbs *s, int limit, hipStream_t st) {
    auto &c = s->coll;
    if (!c.enabled) fail(CMBL_ERR_ARG, "collector not enabled");
    hipLaunchKernelGGL(collector_thin_kernel, dim3((s->W + 63) / 64), dim3(64), 0, st, s->W, c.samp.as<int>(), c.cap,
                       cstate(s, 0), cstate(s, 1), cstate(s, 3), limit);
    HIP_CHECK(hipGetLastError());
}

// the oldest history step any walker's current window reads, and the
// smallest sample count: both must be in range for the window statistics
__global__ void window_first_kernel(int W, const int *samp, int samp_cap, const int *start, const int *count,
                                    int *out)
{
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= W) return;
    const int cnt = count[w];
    atomicMin(&out[1], cnt);
    if (cnt < 2) return;
    atomicMin(&out[0], samp[(size_t)((start[w] + cnt / 2 - 1) % samp_cap) * W + w]);
}

static void check_window_in_ring(cmbs *s) {
    auto &c = s->coll;
    const int init[2] = {0x7fffffff, 0x7fffffff};
    HIP_CHECK(hipMemcpy(c.flag.p, init, 8, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(window_first_kernel, dim3((s->W + 255) / 256), dim3(256), 0, 0, s->W, c.samp.as<int>(), c.cap,
                       cstate(s, 0), cstate(s, 1), c.flag.as<int>());
    HIP_CHECK(hipGetLastError());
    int r[2];
    HIP_CHECK(hipMemcpy(r, c.flag.p, 8, hipMemcpyDeviceToHost));
    if (r[1] < 2) fail(CMBL_ERR_ARG, "a walker has %d samples: too few for a window", r[1]);
    if (s->hist_count - r[0] > s->hist_cap)
        fail(CMBL_ERR_ARG, "a window starts at history step %d, no longer in the ring (count %d, capacity %d): "
                           "enlarge the history", r[0], s->hist_count, s->hist_cap);
}

void chain_moments_launch(const double *means, const double *covs, int W, int n, double count, const int *wcount,
                          const double *gmean, double *out, hipStream_t stream);

void sampler_collector_moments(cmbs *s, const double *gmean, double *out, hipStream_t stream) {
    auto &c = s->coll;
    if (!c.enabled) fail(CMBL_ERR_ARG, "collector not enabled");
    if (!gmean) check_window_in_ring(s);
    const int n = s->n_used;
    s->mom.grow((size_t)s->W * (n + n * n) * 8);
    double *means = s->mom.as<double>(), *covs = means + (size_t)s->W * n;
    if (!gmean) {   // pass 1 computes the per-walker moments; pass 2 reuses them
        const dim3 gm((s->W + 63) / 64), gc((s->W + 63) / 64, n), blk(64 * CPH);
        const double *h = s->hist.as<double>();
        auto run = [&](auto kmean, auto kcov) {
            hipLaunchKernelGGL(kmean, gm, blk, 0, stream, h, s->hist_cap, s->W, n, c.samp.as<int>(), c.cap,
                               cstate(s, 0), cstate(s, 1), means, c.wcount.as<int>());
            HIP_CHECK(hipGetLastError());
            hipLaunchKernelGGL(kcov, gc, blk, 0, stream, h, s->hist_cap, s->W, n, c.samp.as<int>(), c.cap,
                               cstate(s, 0), cstate(s, 1), means, covs);
            HIP_CHECK(hipGetLastError());
        };
        if (n <= 8) run(coll_mean_kernel<8>, coll_cov_kernel<8>);
        else if (n <= 16) run(coll_mean_kernel<16>, coll_cov_kernel<16>);
        else if (n <= 32) run(coll_mean_kernel<32>, coll_cov_kernel<32>);
        else run(coll_mean_kernel<64>, coll_cov_kernel<64>);
    }
    chain_moments_launch(means, covs, s->W, n, 0.0, c.wcount.as<int>(), gmean, out, stream);
}

void sampler_collector_limits(cmbs *s, const int *params, int ncheck, double limfrac, double *out,
                              hipStream_t stream) {
    auto &c = s->coll;
    if (!c.enabled) fail(CMBL_ERR_ARG, "collector not enabled");
    if (ncheck <= 0) return;
    for (int k = 0; k < ncheck; k++)
        if (params[k] < 0 || params[k] >= s->n_used) fail(CMBL_ERR_ARG, "limit parameter %d out of range", params[k]);
    check_window_in_ring(s);
    c.steps.grow((size_t)ncheck * 4);
    HIP_CHECK(hipMemcpyAsync(c.steps.p, params, (size_t)ncheck * 4, hipMemcpyHostToDevice, stream));
    hipLaunchKernelGGL(coll_limits_kernel, dim3(s->W, ncheck), dim3(256), 0, stream, s->hist.as<double>(), s->hist_cap,
                       s->W, s->n_used, c.samp.as<int>(), c.cap, cstate(s, 0), cstate(s, 1), c.steps.as<int>(), ncheck,
                       limfrac, out);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipStreamSynchronize(stream));
}

size_t sampler_collector_bytes(const cmbs *s) {
    return s->coll.enabled ? ((size_t)s->coll.cap + 5 + s->n_used) * s->W * 4 : 0;
}

void sampler_collector_save(cmbs *s, void *buf) {
    HIP_CHECK(hipDeviceSynchronize());
    char *p = static_cast<char *>(buf);
    HIP_CHECK(hipMemcpy(p, s->coll.samp.p, (size_t)s->coll.cap * s->W * 4, hipMemcpyDeviceToHost));
    HIP_CHECK(hipMemcpy(p + (size_t)s->coll.cap * s->W * 4, s->coll.state.p, (size_t)(5 + s->n_used) * s->W * 4,
                        hipMemcpyDeviceToHost));
}

void sampler_collector_load(cmbs *s, const void *buf) {
    HIP_CHECK(hipDeviceSynchronize());
    const char *p = static_cast<const char *>(buf);
    HIP_CHECK(hipMemcpy(s->coll.samp.p, p, (size_t)s->coll.cap * s->W * 4, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(s->coll.state.p, p + (size_t)s->coll.cap * s->W * 4, (size_t)(5 + s->n_used) * s->W * 4,
                        hipMemcpyHostToDevice));
}

}  // namespace cmamd
