// Batched symmetric quadratic form on the f64 MFMA (see quadform.h).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <functional>

#include "quadform.h"
#include "qftile.h"
#include "smallgauss.h"

namespace cmamd {

typedef double f64x4 __attribute__((ext_vector_type(4)));


#ifdef CMAMD_STAMPS
// per-workgroup phase timestamps (s_memtime; instrumented build only, tools/qf_stamps.py):
// start, first tile landed, K loop done, partial + ticket done, end; item nJ,
// partial stored and drained (before the ticket), XCC id
__device__ unsigned long long g_qf_stamps[1024][8];
#define QSTAMP(k)                                                                                  \
    do {                                                                                           \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                               \
        const int b_ = blockIdx.x + blockIdx.y * gridDim.x;                                        \
        if (tid == 0 && b_ < 1024) g_qf_stamps[b_][k] = t_;                                        \
    } while (0)
#else
#define QSTAMP(k) ((void)0)
#endif

// Quadratic form, symmetric split-K.  With Ct = C^-1 whose diagonal 64x64
// blocks are halved,  Delta^T C^-1 Delta / 2 = sum_I Delta_I^T sum_{J>=I} Ct_IJ Delta_J,
// so -lnL needs only the upper block triangle.  A workgroup owns one
// (row block I, column-block range) item for 64 walkers: a double-buffered
// K loop (LDS-DMA fills one BK step ahead) of f64 MFMA 16x16x4 into four
// 16x16 accumulators per wave, then the dot with Delta_I.  Within a BK step
// lane group g = lane>>4 takes k = 8g .. 8g+7 (any k order is valid as long
// as A and B agree), so each lane reads its fragments as ds_read_b128.
// Partials are handed off in-launch: the last workgroup of each walker tile
// (agent-scope release / ticket / acquire, cdna_hip_programming.md section 5
// split-K recipe) sums them in fixed item order: deterministic results.
// Without TICKET the partials are only stored: the consumer kernel that runs
// next on the stream combines them (QFDeferred), with no in-launch hand-off.
template <bool TICKET>
__device__ __forceinline__ void quadform_body(
    double *smem, int item_ix, int tile,
    const double *__restrict__ Ct, int Np, const double *__restrict__ delta, int W,
    const QFItem *__restrict__ items, int n_items,
    double *__restrict__ partial, unsigned int *__restrict__ counters, const double *__restrict__ addend,
    double *__restrict__ out, const int *__restrict__ wcount)
{
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int li = lane & 15, lk = lane >> 4;
    QSTAMP(0);
    const int w0 = tile * QF_TILE;
    if (wcount) {                                     // sparse evaluation: walkers [0, *wcount) live
        const int wc = *wcount;
        if (w0 >= wc) return;                         // the whole tile: no ticket taken
        W = min(W, wc);
    }
    const QFItem it = items[item_ix];
    const int nsteps = it.nJ * (QF_TILE / BK);
    const int kbase0 = it.J0 * QF_TILE;
    const double *Arow = Ct + (size_t)(it.I * QF_TILE) * Np;      // rows of the I panel
    const double *Brow = delta + (size_t)w0 * Np;               // walker rows of the tile

    f64x4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; t++) acc[t] = f64x4{0.0, 0.0, 0.0, 0.0};
    // the epilogue's Delta_I tile is loaded during the last K step (issued
    // behind that step's barrier, so the first tiles' wait does not include it)
    double2 dI[QF_TILE * QF_TILE / 2 / 256];
    dma_tile(smem, Arow, Np, kbase0, wave, lane);
    dma_tile(smem + QF_TILE * BK, Brow, Np, kbase0, wave, lane);
    for (int s = 0; s < nsteps; s++) {
        const int buf = s & 1;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();                              // tile s landed for every wave; buf^1 free
        if (s == 0) QSTAMP(1);
        if (s + 1 < nsteps) {
            double *nb = smem + (buf ^ 1) * 2 * QF_TILE * BK;
            dma_tile(nb, Arow, Np, kbase0 + (s + 1) * BK, wave, lane);
            dma_tile(nb + QF_TILE * BK, Brow, Np, kbase0 + (s + 1) * BK, wave, lane);
        } else {
#pragma unroll
            for (int u = 0; u < QF_TILE * QF_TILE / 2 / 256; u++) {
                const int e = tid + 256 * u, r = e >> 5, c2 = (e & 31) * 2;
                dI[u] = *reinterpret_cast<const double2 *>(delta + (size_t)(w0 + r) * Np + it.I * QF_TILE + c2);
            }
        }
        const double *A = smem + buf * 2 * QF_TILE * BK;
        const double *B = A + QF_TILE * BK;
        double2 a[4][4], b[4];
        {
            const int r = 16 * wave + li;
#pragma unroll
            for (int q = 0; q < 4; q++)
                b[q] = *reinterpret_cast<const double2 *>(B + r * BK + (((lk * 4 + q) ^ swz(r)) * 2));
        }
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const int r = 16 * t + li;
#pragma unroll
            for (int q = 0; q < 4; q++)
                a[t][q] = *reinterpret_cast<const double2 *>(A + r * BK + (((lk * 4 + q) ^ swz(r)) * 2));
        }
        // consecutive MFMAs go to different accumulators (dependency distance 4);
        // each accumulator still sums k in the same order
#pragma unroll
        for (int q = 0; q < 4; q++) {
#pragma unroll
            for (int t = 0; t < 4; t++)
                acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[t][q].x, b[q].x, acc[t], 0, 0, 0);
#pragma unroll
            for (int t = 0; t < 4; t++)
                acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[t][q].y, b[q].y, acc[t], 0, 0, 0);
        }
    }
    __syncthreads();                                  // all waves done with the operand buffers
    QSTAMP(2);
#ifdef CMAMD_STAMPS
    if (tid == 0 && blockIdx.x + blockIdx.y * gridDim.x < 1024) {
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        g_qf_stamps[blockIdx.x + blockIdx.y * gridDim.x][5] = it.nJ;
        g_qf_stamps[blockIdx.x + blockIdx.y * gridDim.x][7] = xcc & 15;
    }
#endif
    // Delta_I tile: smem[n][i] (row stride QF_TILE+2)
#pragma unroll
    for (int u = 0; u < QF_TILE * QF_TILE / 2 / 256; u++) {
        const int e = tid + 256 * u, r = e >> 5, c2 = (e & 31) * 2;
        const double2 v = (w0 + r < W) ? dI[u] : make_double2(0.0, 0.0);
        *reinterpret_cast<double2 *>(smem + r * (QF_TILE + 2) + c2) = v;
    }
    __syncthreads();
    // f64 16x16x4 C/D layout: col = lane&15 (walker n), row = (lane>>4) + 4*r (i)
    const int n = 16 * wave + li;
    double sacc = 0.0;
#pragma unroll
    for (int t = 0; t < 4; t++)
#pragma unroll
        for (int r = 0; r < 4; r++) sacc += acc[t][r] * smem[n * (QF_TILE + 2) + 16 * t + lk + 4 * r];
    sacc += __shfl_xor(sacc, 16);
    sacc += __shfl_xor(sacc, 32);
    double *tile_part = partial + (size_t)tile * n_items * QF_TILE;
    if (!TICKET) {                                    // the kernel boundary publishes them
        if (lk == 0) tile_part[(size_t)item_ix * QF_TILE + n] = sacc;
        return;
    }
    // ---- in-launch hand-off of the tile's partials to its last-arriving workgroup
    // (cdna_hip_programming.md section 5 split-K recipe, write-through form): the
    // partials are stored sc1 (agent-scope relaxed atomic stores), drained by
    // every storing wave, then one relaxed ticket; no release fence, so no L2
    // write-back of the tile's other dirty lines
    if (lk == 0)
        __hip_atomic_store(tile_part + (size_t)item_ix * QF_TILE + n, sacc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    QSTAMP(6);
    unsigned int *flag = reinterpret_cast<unsigned int *>(smem + 64 * (QF_TILE + 2));
    if (tid == 0) {
        const unsigned int t = __hip_atomic_fetch_add(counters + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        flag[0] = (t == (unsigned int)n_items - 1u) ? 1u : 0u;
    }
    __syncthreads();
    QSTAMP(3);
    if (flag[0] == 0u) return;
    if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    // the fixed combine order of quadform.h: wave q takes groups q, q+4, q+8, q+12
    double *red = smem + 64 * (QF_TILE + 2) + 8;
#pragma unroll
    for (int j = 0; j < QF_GROUPS / 4; j++) {
        const int g = wave + 4 * j;
        red[g * QF_TILE + lane] = qf_group_sum(tile_part, n_items, g, lane);
    }
    __syncthreads();
    if (tid < QF_TILE) {
        const double v = qf_tree(red + lane, QF_TILE);
        if (w0 + lane < W) out[w0 + lane] = addend ? v + addend[w0 + lane] : v;
        if (lane == 0) counters[tile] = 0u;
    }
    QSTAMP(4);
}

template <bool TICKET>
__global__ __launch_bounds__(256, 2) void quadform_ksplit(
    const double *__restrict__ Ct, int Np, const double *__restrict__ delta, int W,
    const QFItem *__restrict__ items, int n_items, int xcd_map,
    double *__restrict__ partial, unsigned int *__restrict__ counters, const double *__restrict__ addend,
    double *__restrict__ out, const int *__restrict__ wcount)
{
    __shared__ __attribute__((aligned(16))) double smem[QF_LDS_DOUBLES];
    int item_ix, tile;
    qf_place(blockIdx.x + blockIdx.y * gridDim.x, n_items, xcd_map, item_ix, tile);
    quadform_body<TICKET>(smem, item_ix, tile, Ct, Np, delta, W, items, n_items, partial, counters, addend, out,
                          wcount);
}

// The deferred quadratic form with a small gaussian chi^2 riding along: the
// first workgroups are quadform_ksplit<false>'s in its order, the last ns run
// smallgauss.h's body over the co-run's walkers.  One launch instead of two on
// the sampler's critical path, and the chi^2 workgroups fill the slots the
// quadratic form leaves free (480 of 512 at W = 1024) and those its one-block
// items release half way (MI355X, plik_lite + lensing, W = 1024: 15.4 us
// against 13.5 + 4.6 us for the two launches; with the chi^2 workgroups first
// 19.8 us, with 8 walkers per chi^2 workgroup 16.5 us).  Both bodies compute
// exactly what their own kernels do.
template <int WT>
__global__ __launch_bounds__(256, 2) void quadform_corun(
    const double *__restrict__ Ct, int Np, const double *__restrict__ delta, int W,
    const QFItem *__restrict__ items, int n_items, int xcd_map, double *__restrict__ partial,
    SmallGaussLaunch co, int ns, int nq)
{
    static_assert(small_gauss_lds_doubles<WT>() <= QF_LDS_DOUBLES, "co-run LDS");
    __shared__ __attribute__((aligned(16))) double smem[QF_LDS_DOUBLES];
    // the chi^2 workgroups start at a multiple of 8, so small_gauss_group's
    // lb % 8 is the XCD (blockIdx.x % 8); workgroups nq .. nqp - 1 are padding
    const int nqp = (nq + 7) & ~7;
    const int b = blockIdx.x;
    if (b >= nqp) {
        const int q = small_gauss_group(b - nqp, ns);
        if (q < ns) small_gauss_body<WT>(co, smem, q);
        return;
    }
    if (b >= nq) return;
    int item_ix, tile;
    qf_place(b, n_items, xcd_map, item_ix, tile);
    quadform_body<false>(smem, item_ix, tile, Ct, Np, delta, W, items, n_items, partial, nullptr, nullptr, nullptr,
                         nullptr);
}

#ifdef CMAMD_STAMPS
extern "C" int cmamd_debug_qf_stamps(unsigned long long *host) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_qf_stamps), sizeof(g_qf_stamps)) == hipSuccess ? 0 : -5;
}
#endif


// ------------------------------------------------------------------ host side

void QuadForm::init(const std::vector<double> &M, int n_) {
    n = n_;
    Np = (n + QF_TILE - 1) / QF_TILE * QF_TILE;
    nblk = Np / QF_TILE;
    // Ct: M padded to Np with the diagonal 64x64 blocks halved (exact: x0.5), so
    // x^T M x / 2 = sum_I x_I^T sum_{J>=I} Ct_IJ x_J needs only the upper block triangle
    std::vector<double> ct((size_t)Np * Np, 0.0);
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) {
            const double v = M[(size_t)i * n + j];
            ct[(size_t)i * Np + j] = (i / QF_TILE == j / QF_TILE) ? 0.5 * v : v;
        }
    d_ct.alloc(ct.size() * 8);
    d_ct.upload(ct.data(), ct.size() * 8);
    for (int kb = 1; kb <= MAXKB; kb++) {
        items[kb].clear();
        for (int I = 0; I < nblk; I++)
            for (int J0 = I; J0 < nblk; J0 += kb) items[kb].push_back(QFItem{I, J0, std::min(kb, nblk - J0), 0});
        d_items[kb].alloc(items[kb].size() * sizeof(QFItem));
        d_items[kb].upload(items[kb].data(), items[kb].size() * sizeof(QFItem));
    }
    kb_for_tiles.clear();
}

size_t QuadForm::nmax_items() const {
    size_t nmax = 0;
    for (int kb = 1; kb <= MAXKB; kb++) nmax = std::max(nmax, items[kb].size());
    return nmax;
}

size_t QuadForm::workspace_size(int W) const {
    const size_t Wp = (size_t)wpad(W), tiles = Wp / QF_TILE;
    return (Wp * Np + tiles * nmax_items() * QF_TILE) * sizeof(double) + ((tiles * 4 + 255) & ~size_t(255));
}

unsigned int *QuadForm::counters(void *ws, int W) const {
    const size_t Wp = (size_t)wpad(W), tiles = Wp / QF_TILE;
    return reinterpret_cast<unsigned int *>(static_cast<double *>(ws) + Wp * Np + tiles * nmax_items() * QF_TILE);
}

// Column-block chunk per work item: the largest chunk whose longest-first
// greedy schedule over 2 workgroups/CU x 256 CUs is (near) the fastest,
// counting a fixed per-workgroup overhead of half a block.  The chunk is
// chosen once per matrix, for 16 walker tiles (W = 1024), not per launch:
// the items fix the order in which a walker's sum is formed, so one choice
// for every walker count keeps each walker's -lnL independent of how many
// walkers share the launch (a walker group, a compacted change-mask slot
// list or a single walker give the same bits).
int QuadForm::choose_kb(int /*tiles*/) {
    const int tiles = 16;
    auto itk = kb_for_tiles.find(tiles);
    if (itk != kb_for_tiles.end()) return itk->second;
    const int slots = 512;
    int best_kb = 1;
    double best = 1e300;
    for (int kb = 1; kb <= MAXKB; kb++) {
        std::vector<double> load(slots, 0.0);
        std::vector<double> jobs;
        for (auto &x : items[kb])
            for (int t = 0; t < tiles; t++) jobs.push_back(x.nJ + 0.5);
        std::sort(jobs.begin(), jobs.end(), std::greater<double>());
        for (double j : jobs) *std::min_element(load.begin(), load.end()) += j;
        const double makespan = *std::max_element(load.begin(), load.end()) + 0.02 * items[kb].size();
        if (makespan < best * 0.98) {
            best = makespan;
            best_kb = kb;
        }
    }
    if (const char *e = std::getenv("CMAMD_QF_KB")) {   // A/B: a fixed chunk (1 .. QF_MAXKB)
        const int k = std::atoi(e);
        if (k >= 1 && k <= MAXKB) best_kb = k;
    }
    kb_for_tiles[tiles] = best_kb;
    return best_kb;
}

void QuadForm::launch(int W, void *ws, const double *addend, double *out, hipStream_t stream, const char *prof_name,
                      const int *wcount) {
    const int tiles = wpad(W) / QF_TILE;
    const int kb = choose_kb(tiles);
    const int n_items = (int)items[kb].size();
    double *x = x_rows(ws);
    double *partial = x + (size_t)wpad(W) * Np;
    unsigned int *cnt = counters(ws, W);
    timed_launch(prof_name, stream, [&](hipEvent_t e0, hipEvent_t e1) {
        hipExtLaunchKernelGGL(quadform_ksplit<true>, dim3(n_items, tiles), dim3(256), 0, stream, e0, e1, 0,
                              d_ct.as<double>(), Np, (const double *)x, W, d_items[kb].as<QFItem>(), n_items,
                              (int)(tiles % 8 == 0), partial, cnt, addend, out, wcount);
    });
    HIP_CHECK(hipGetLastError());
}

QFDeferred QuadForm::launch_deferred(int W, void *ws, const double *addend, hipStream_t stream, const char *prof_name,
                                     const SmallGaussLaunch *co, const char *co_prof_name) {
    const int tiles = wpad(W) / QF_TILE;
    const int kb = choose_kb(tiles);
    const int n_items = (int)items[kb].size();
    double *x = x_rows(ws);
    double *partial = x + (size_t)wpad(W) * Np;
    if (co) {
        const int ns = (co->W + SMALL_WT - 1) / SMALL_WT;
        timed_launch(co_prof_name, stream, [&](hipEvent_t e0, hipEvent_t e1) {
            const int nq = n_items * tiles;
            hipExtLaunchKernelGGL(quadform_corun<SMALL_WT>, dim3(((nq + 7) & ~7) + small_gauss_blocks(ns)), dim3(256),
                                  0, stream, e0, e1, 0,
                                  d_ct.as<double>(), Np, (const double *)x, W, d_items[kb].as<QFItem>(), n_items,
                                  (int)(tiles % 8 == 0), partial, *co, ns, nq);
        });
    } else
    timed_launch(prof_name, stream, [&](hipEvent_t e0, hipEvent_t e1) {
        hipExtLaunchKernelGGL(quadform_ksplit<false>, dim3(n_items, tiles), dim3(256), 0, stream, e0, e1, 0,
                              d_ct.as<double>(), Np, (const double *)x, W, d_items[kb].as<QFItem>(), n_items,
                              (int)(tiles % 8 == 0), partial, (unsigned int *)nullptr, (const double *)nullptr,
                              (double *)nullptr, (const int *)nullptr);
    });
    HIP_CHECK(hipGetLastError());
    QFDeferred d;
    d.partial = partial;
    d.n_items = n_items;
    d.addend = addend;
    return d;
}

QFSource QuadForm::source(int W, void *ws, const double *X) {
    const int tiles = wpad(W) / QF_TILE;
    const int kb = choose_kb(tiles);
    QFSource q;
    q.Ct = d_ct.as<double>();
    q.Np = Np;
    q.xcd_map = (int)(tiles % 8 == 0);
    q.items = d_items[kb].as<QFItem>();
    q.n_items = (int)items[kb].size();
    q.partial = x_rows(ws) + (size_t)wpad(W) * Np;
    q.X = X;
    q.delta = x_rows(ws);
    q.counters = counters(ws, W);
    q.n_counters = n_counters(W);
    return q;
}

// Two evaluations' quadratic forms (the dragging steps' end and start points,
// each on its own workspace) with the in-launch combine, and their small
// gaussian chi^2s riding along: [quadratic form a][quadratic form b][chi^2 a]
// [chi^2 b] (set b absent: nq_b = 0 and no chi^2 b).  The tickets must be zero at launch (the pass zeroes them:
// theory_window_pair); each tile's last arriver leaves its ticket zero again.
template <int WT>
__global__ __launch_bounds__(256, 2) void quadform_pair_ticket(QFSource qa, double *out_a, QFSource qb, double *out_b,
                                                               int W, int nq, SmallGaussLaunch ga, SmallGaussLaunch gb,
                                                               int ng, int nq_b)
{
    static_assert(small_gauss_lds_doubles<WT>() <= QF_LDS_DOUBLES, "co-run LDS");
    __shared__ __attribute__((aligned(16))) double smem[QF_LDS_DOUBLES];
    int b = blockIdx.x;
    if (b < nq + nq_b) {
        const bool second = b >= nq;
        const QFSource &q = second ? qb : qa;
        int item_ix, tile;
        qf_place(b - (second ? nq : 0), q.n_items, q.xcd_map, item_ix, tile);
        quadform_body<true>(smem, item_ix, tile, q.Ct, q.Np, q.delta, W, q.items, q.n_items, q.partial, q.counters,
                            nullptr, second ? out_b : out_a, nullptr);
        return;
    }
    b -= (nq + nq_b + 7) & ~7;   // the chi^2 workgroups start at a multiple of 8 (small_gauss_group's XCD)
    if (b < 0) return;
    const int gp = small_gauss_blocks(ng);
    const int q = small_gauss_group(b < gp ? b : b - gp, ng);
    if (q < ng) small_gauss_body<WT>(b < gp ? ga : gb, smem, q);
}

void launch_qf_pair(const QFSource &qa, double *out_a, const QFSource *qb, double *out_b, int W,
                    const SmallGaussLaunch *ga, const SmallGaussLaunch *gb, hipStream_t stream, const char *prof_name) {
    if (!qa.delta || (qb && (qb->n_items != qa.n_items || !qb->delta))) fail(CMBL_ERR_ARG, "internal: quadratic-form pair");
    const int nq = qa.n_items * (QuadForm::wpad(W) / QF_TILE);
    const int ng = ga ? (W + SMALL_WT - 1) / SMALL_WT : 0;
    const SmallGaussLaunch none{};
    // one set: [quadratic form a][chi^2 a]
    const int nq_b = qb ? nq : 0, ng_b = gb ? ng : 0;
    const dim3 grid(((nq + nq_b + 7) & ~7) + small_gauss_blocks(ng) + small_gauss_blocks(ng_b));
    timed_launch(prof_name, stream, [&](hipEvent_t e0, hipEvent_t e1) {
        hipExtLaunchKernelGGL(quadform_pair_ticket<SMALL_WT>, grid, dim3(256), 0, stream, e0, e1, 0, qa, out_a,
                              qb ? *qb : qa, out_b, W, nq, ga ? *ga : none, gb ? *gb : none, ng, nq_b);
    });
    HIP_CHECK(hipGetLastError());
}

// Cholesky inverse of an SPD matrix (Matrix_Inverse: dpotrf 'L' + dpotri,
// source/Matrix_utils_new.f90:1478-1569), row-major, in place.
void spd_inverse(std::vector<double> &A, int n) {
    for (int i = 0; i < n; i++)
        if (std::fabs(A[(size_t)i * n + i]) < 1e-30) fail(CMBL_ERR_NUMERIC, "Matrix_Inverse: very small diagonal");
    for (int j = 0; j < n; j++) {
        double d = A[(size_t)j * n + j];
        for (int k = 0; k < j; k++) d -= A[(size_t)j * n + k] * A[(size_t)j * n + k];
        if (!(d > 0.0)) fail(CMBL_ERR_NUMERIC, "Matrix_Inverse: covariance not positive definite (%d)", j + 1);
        d = std::sqrt(d);
        A[(size_t)j * n + j] = d;
        for (int i = j + 1; i < n; i++) {
            double s = A[(size_t)i * n + j];
            for (int k = 0; k < j; k++) s -= A[(size_t)i * n + k] * A[(size_t)j * n + k];
            A[(size_t)i * n + j] = s / d;
        }
    }
    for (int j = 0; j < n; j++) {           // L^-1, lower
        A[(size_t)j * n + j] = 1.0 / A[(size_t)j * n + j];
        for (int i = j + 1; i < n; i++) {
            double s = 0.0;
            for (int k = j; k < i; k++) s += A[(size_t)i * n + k] * A[(size_t)k * n + j];
            A[(size_t)i * n + j] = -s / A[(size_t)i * n + i];
        }
    }
    std::vector<double> T((size_t)n * n);
    for (int i = 0; i < n; i++)
        for (int j = 0; j <= i; j++) {
            double s = 0.0;
            for (int k = i; k < n; k++) s += A[(size_t)k * n + i] * A[(size_t)k * n + j];
            T[(size_t)i * n + j] = s;
            T[(size_t)j * n + i] = s;
        }
    A.swap(T);
}


// Symmetric eigen-decomposition by cyclic Jacobi (host; data-set set-up only):
// evals ascending, evecs row-major with eigenvector k in column k, as
// Matrix_Diagonalize (DSYEV 'V', source/Matrix_utils_new.f90:361-383).
void sym_eigen(std::vector<double> A, int n, std::vector<double> &evals, std::vector<double> &evecs) {
    std::vector<double> V((size_t)n * n, 0.0);
    for (int i = 0; i < n; i++) V[(size_t)i * n + i] = 1.0;
    for (int sweep = 0; sweep < 100; sweep++) {
        double off = 0.0, tot = 0.0;
        for (int i = 0; i < n; i++)
            for (int j = 0; j < n; j++) {
                const double a = A[(size_t)i * n + j] * A[(size_t)i * n + j];
                tot += a;
                if (i != j) off += a;
            }
        if (off <= 1e-32 * tot || off == 0.0) break;
        for (int p = 0; p < n - 1; p++)
            for (int q = p + 1; q < n; q++) {
                const double apq = A[(size_t)p * n + q];
                if (apq == 0.0) continue;
                const double app = A[(size_t)p * n + p], aqq = A[(size_t)q * n + q];
                const double theta = (aqq - app) / (2.0 * apq);
                const double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
                const double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < n; k++) {    // A <- A J
                    const double akp = A[(size_t)k * n + p], akq = A[(size_t)k * n + q];
                    A[(size_t)k * n + p] = c * akp - s * akq;
                    A[(size_t)k * n + q] = s * akp + c * akq;
                }
                for (int k = 0; k < n; k++) {    // A <- J^T A
                    const double apk = A[(size_t)p * n + k], aqk = A[(size_t)q * n + k];
                    A[(size_t)p * n + k] = c * apk - s * aqk;
                    A[(size_t)q * n + k] = s * apk + c * aqk;
                }
                A[(size_t)p * n + q] = A[(size_t)q * n + p] = 0.0;
                for (int k = 0; k < n; k++) {    // V <- V J
                    const double vkp = V[(size_t)k * n + p], vkq = V[(size_t)k * n + q];
                    V[(size_t)k * n + p] = c * vkp - s * vkq;
                    V[(size_t)k * n + q] = s * vkp + c * vkq;
                }
            }
    }
    std::vector<int> ord(n);
    for (int i = 0; i < n; i++) ord[i] = i;
    std::sort(ord.begin(), ord.end(), [&](int a, int b) { return A[(size_t)a * n + a] < A[(size_t)b * n + b]; });
    evals.resize(n);
    evecs.assign((size_t)n * n, 0.0);
    for (int k = 0; k < n; k++) {
        evals[k] = A[(size_t)ord[k] * n + ord[k]];
        for (int i = 0; i < n; i++) evecs[(size_t)i * n + k] = V[(size_t)i * n + ord[k]];
    }
}

// M <- U D^pw U^T  (Matrix_Root, source/Matrix_utils_new.f90:421-440)
void sym_power(std::vector<double> &A, int n, double pw) {
    std::vector<double> d, U;
    sym_eigen(A, n, d, U);
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) {
            double s = 0.0;
            for (int k = 0; k < n; k++) s += U[(size_t)i * n + k] * std::pow(d[k], pw) * U[(size_t)j * n + k];
            A[(size_t)i * n + j] = s;
        }
}

}  // namespace cmamd
