// Batched Metropolis sampler: W independent CosmoMC chains, one per walker
// (one GPU lane per walker for the sequential per-chain logic), with the
// likelihoods evaluated as batched kernels over all walkers in between.
//
// Per-walker semantics follow the reference exactly, including the random
// number call order, so that walker w with RANMAR seeds (ij_w, kl_w)
// reproduces a reference chain started with the same seeds:
//   RANMAR / Gaussian1 / randexp1 / RandIndices / RandRotationD  RandUtils.f90:93-374
//   BlockedProposer GetProposal{,Fast,Slow}, ProposeVec, Propose_r,
//   UpdateParams, CyclicIndexRandomizer%Next                      propose.f90:75-298
//   GetLogLike = bounds + like/T + priors/T                        calclike.f90:82-151
//   MetropolisAccept, MoveDone multiplicity                        MCMC.f90:119-190
//
// The chain logic is a long chain of dependent state reads (RNG index ->
// RNG table -> block cycle -> rotation -> mapping ...).  Served from HBM each
// would cost a memory round trip; instead mh_kernel stages the whole
// per-walker state (sampler.h Rows) and the shared tables into LDS with
// independent coalesced loads, runs the chain out of LDS and writes back.
#include <algorithm>
#include <cmath>
#include <cstring>

#include <cstdlib>

#include "plikbin.h"
#include "qfs_body.h"
#include "quadform.h"
#include "sampler.h"
#include "smallgauss.h"
#ifdef CMAMD_STAMPS
namespace cmamd {
// mh_step_kernel (tools/uni_stamps.py), [0] the middle launches, [1] the last
// (accept-only) launch: start, the Metropolis wait's end, XCC id, end, role + 1
__device__ unsigned long long g_uni_stamps[2][2048][6];   // start, wait done, xcc, end, role + 1, folded chi^2 done
}
#endif
#include "theorypass_body.h"

namespace cmamd {

static constexpr double LOGZERO = CMBL_LOGZERO;
static constexpr int MAXP = 64;        // max parameters per chain
static constexpr int MAXBLK = 32;      // max block size
static constexpr int NB = 64;          // walker tile of the history / collector kernels (one wavefront)
// mh_kernel: MB walkers per block (lanes 0..MB-1 of wave 0 run their chain
// logic) and MH_THREADS threads, i.e. NV = MH_THREADS / MB groups of MB threads
// for the staging, the deferred combines and the multi-group products.  With
// 16-walker blocks a W = 1024 step spreads over 64 CUs instead of 16: each
// block stages a quarter of the state image (round 3: 64-walker blocks, 16
// waves, 12.9 us).
#ifndef CMAMD_MB
#define CMAMD_MB 16
#endif
static constexpr int MB = CMAMD_MB;
static constexpr int MH_THREADS = 256;
static constexpr int NV = MH_THREADS / MB;
static_assert(NV >= QF_GROUPS && NV % QF_GROUPS == 0, "a group per split-K group sum");
static_assert(64 % MB == 0, "blocks tile the 64-walker rows of the split-K partials");

// strided per-walker column view (LDS: stride MB; HBM: stride W)
template <class T> struct Col {
    T *p;
    int s;
    __device__ T &operator[](int i) const { return p[(size_t)i * s]; }
};

// ------------------------------------------------------------ RNG (RandUtils.f90)

struct Rng {
    Col<double> u;  // u(1:97)
    double c;
    int i97, j97, iset;
    double gset;
    int nd = 0;     // draws so far (the lean chain writes back the ring entries they overwrote)
};

__device__ __forceinline__ double ranmar(Rng &r)
{   // RandUtils.f90:350-374
    double uni = r.u[r.i97 - 1] - r.u[r.j97 - 1];
    if (uni < 0.0) uni += 1.0;
    r.u[r.i97 - 1] = uni;
    if (--r.i97 == 0) r.i97 = 97;
    if (--r.j97 == 0) r.j97 = 97;
    r.nd++;
    const double cd = 7654321.0 / 16777216.0, cm = 16777213.0 / 16777216.0;
    r.c -= cd;
    if (r.c < 0.0) r.c += cm;
    uni -= r.c;
    if (uni < 0.0) uni += 1.0;
    return uni;
}

__device__ __forceinline__ double gaussian1(Rng &r)
{   // RandUtils.f90:156-178
    if (r.iset == 0) {
        double v1, v2, rr;
        do {
            v1 = 2.0 * ranmar(r) - 1.0;
            v2 = 2.0 * ranmar(r) - 1.0;
            rr = v1 * v1 + v2 * v2;
        } while (rr >= 1.0);
        const double fac = sqrt(-2.0 * log(rr) / rr);
        r.gset = v1 * fac;
        r.iset = 1;
        return v2 * fac;
    }
    r.iset = 0;
    return r.gset;
}

__device__ __forceinline__ float randexp1(Rng &r)
{   // RandUtils.f90:189-233, REAL(4) arithmetic (built with -ffp-contract=off)
    const float alog2 = 0.6931471805599453f, a = 5.7133631526454228f, b = 3.4142135623730950f;
    const float c = -1.6734053240284925f, p = 0.9802581434685472f, aa = 5.6005707569738080f;
    const float bb = 3.3468106480569850f, hh = 0.0026106723602095f, dd = 0.0857864376269050f;
    float u = (float)ranmar(r);
    while (u <= 0.0f) u = (float)ranmar(r);
    float g = c;
    u = u + u;
    while (u < 1.0f) {
        g = g + alog2;
        u = u + u;
    }
    u = u - 1.0f;
    if (u <= p) return g + aa / (bb - u);
    for (;;) {
        u = (float)ranmar(r);
        const float y = a / (b - u);
        const float up = (float)ranmar(r);
        const float bu = b - u;
        if ((up * hh + dd) * (bu * bu) <= expf(-(y + c))) return g + y;
    }
}

__global__ void rng_init_kernel(DevCfg c, const int *ij, const int *kl)
{   // RMARIN, RandUtils.f90:286-348
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= c.W) return;
    const size_t W = c.ld;
    int i = (ij[w] / 177) % 177 + 2, j = ij[w] % 177 + 2, k = (kl[w] / 169) % 178 + 1, l = kl[w] % 169;
    for (int ii = 0; ii < 97; ii++) {
        double s = 0.0, t = 0.5;
        for (int jj = 0; jj < 24; jj++) {
            const int m = (((i * j) % 179) * k) % 179;
            i = j;
            j = k;
            k = m;
            l = (53 * l + 1) % 169;
            if ((l * m) % 64 >= 32) s += t;
            t *= 0.5;
        }
        c.sd[(c.rows.U + ii) * W + w] = s;
    }
    c.sd[c.rows.C * W + w] = 362436.0 / 16777216.0;
    c.sd[c.rows.G * W + w] = 0.0;
    c.si[c.rows.I97 * W + w] = 97;
    c.si[c.rows.J97 * W + w] = 33;
    c.si[c.rows.ISET * W + w] = 0;
}

// ------------------------------------------------------------ per-walker view

struct Tabs {   // shared tables (LDS copies)
    const int *ti;   // the whole int table (likelihood nuisance_indices at DevCfg::like_nidx offsets)
    const int *blk_n, *blk_nchanged, *blk_changed_off, *blk_map_off, *blk_R_off, *changed, *pfi, *params_used;
    const double *mapping, *pmin, *pmax, *pmean, *pstd, *lin_w, *lin_m, *lin_s, *covinv, *center;
};

// td_cov: where the test-Gaussian tables (covinv, center: the tail of the
// double table) live -- the LDS copy, or tab_d itself when not staged
__device__ Tabs make_tabs(const DevCfg &c, const int *ti, const double *td, const double *td_cov = nullptr)
{
    const TabLayout &l = c.tl;
    if (!td_cov) td_cov = td;
    return Tabs{ti, ti + l.blk_n, ti + l.blk_nchanged, ti + l.blk_changed_off, ti + l.blk_map_off, ti + l.blk_R_off,
                ti + l.changed, ti + l.pfi, ti + l.params_used, td + l.mapping, td + l.pmin, td + l.pmax,
                td + l.pmean, td + l.pstd, td + l.lin_w, td + l.lin_m, td + l.lin_s, td_cov + l.covinv,
                td_cov + l.center};
}

struct Walker {
    Rng r;
    Col<double> R, P, trial, vec;
    Col<int> cyc, cyclp, blklp, itmp;
    int fast_ix;
    int defer = 0;    // leave the mapping product to the caller (block index in pend_b, vec filled)
    int pend_b = -1;
    int defer_rot = 0;   // leave a new rotation of a wide block to rot_kernel (block index in pend_rot)
    int pend_rot = -1;
    double r1 = 0.0;     // a one-parameter block's rotation, just drawn (R may live in HBM: no read-back)
    int col_pre = 0;     // vec already holds the proposal's column of R (mh_body's pre_col)
};

__device__ int cyc_next(Walker &k, int which, int n, int base)
{   // CyclicIndexRandomizer%Next, propose.f90:75-86 (RandIndices RandUtils.f90:93-108)
    const int lp = k.cyclp[which] % n + 1;
    k.cyclp[which] = lp;
    if (lp == 1) {
        if (n == 1) {
            (void)ranmar(k.r);                      // ix = int(ranmar()*1)+1 = 1
            k.cyc[base] = 1;
        } else {
            for (int i = 0; i < n; i++) k.itmp[i] = i + 1;
            for (int i = 1; i <= n; i++) {
                const int ix = (int)(ranmar(k.r) * (n + 1 - i)) + 1;
                k.cyc[base + i - 1] = k.itmp[ix - 1];
                k.itmp[ix - 1] = k.itmp[n + 1 - i - 1];
            }
        }
    }
    return k.cyc[base + lp - 1];
}

// Rows of R may live in HBM (blocks too big for the LDS image): every pass over
// a row loads it RCH elements at a time, all in flight together, instead of one
// dependent round trip per element.  The sums keep the reference's q order.
static constexpr int RCH = 8;

__device__ void rot_matrix(Walker &k, int off, int n)
{   // RotMatrix propose.f90:88-102 -> RandRotationD RandUtils.f90:133-153
    // element (j,i) (row j) of this block's R at R[off + j*n + i]
    if (n > 1) {
        for (int j = 0; j < n; j++) {
            double norm;
            for (;;) {
                for (int i = 0; i < n; i++) k.vec[i] = gaussian1(k.r);
                for (int i = 0; i < j; i++) {   // vec = vec - sum(vec*R(i,:))*R(i,:)
                    const int base = off + i * n;
                    double s = 0.0;
                    for (int q0 = 0; q0 < n; q0 += RCH) {
                        double rv[RCH], vv[RCH];
#pragma unroll
                        for (int u = 0; u < RCH; u++) {
                            const int q = q0 + u;
                            rv[u] = q < n ? k.R[base + q] : 0.0;
                            vv[u] = q < n ? k.vec[q] : 0.0;
                        }
#pragma unroll
                        for (int u = 0; u < RCH; u++)
                            if (q0 + u < n) s += vv[u] * rv[u];
                    }
                    for (int q0 = 0; q0 < n; q0 += RCH) {
                        double rv[RCH];
#pragma unroll
                        for (int u = 0; u < RCH; u++) rv[u] = q0 + u < n ? k.R[base + q0 + u] : 0.0;
#pragma unroll
                        for (int u = 0; u < RCH; u++)
                            if (q0 + u < n) k.vec[q0 + u] = k.vec[q0 + u] - s * rv[u];
                    }
                }
                norm = 0.0;
                for (int q = 0; q < n; q++) norm += k.vec[q] * k.vec[q];
                if (norm > 1e-3) break;
            }
            const double sn = sqrt(norm), rsn = 1.0 / sn;
            for (int q = 0; q < n; q++) k.R[off + j * n + q] = div_rn(k.vec[q], sn, rsn);   // = vec(q) / sn
        }
    } else {
        for (int i = 0; i < n * n; i++) k.R[off + i] = 0.0;
        for (int i = 0; i < n; i++) {
            k.r1 = (ranmar(k.r) - 0.5) >= 0.0 ? 1.0 : -1.0;
            k.R[off + i * n + i] = k.r1;
        }
    }
}

// blocks this wide get their rotations from rot_kernel.  (Narrower ones stay
// in the chain: config5_bk15_plik's 7-wide foreground block deferred measured
// mh_kernel 34.2 -> 20.7 us plus rot_kernel 15.0 us a step, no gain.)
static constexpr int ROT_DEFER_MIN = 8;

__device__ void proposal_tail(const DevCfg &c, const Tabs &t, Walker &k, int b, int lp);
__device__ void proposal_r(const DevCfg &c, const Tabs &t, Walker &k, int b, int n, double r1);

__device__ __forceinline__ void block_proposal(const DevCfg &c, const Tabs &t, Walker &k, int bi /*1-based*/)
{   // GetBlockProposal :247-254 -> ProposeVec :105-120 -> Propose_r :122-139 -> UpdateParams :142-149
    const int b = bi - 1;
    const int n = t.blk_n[b];
    const int off = t.blk_R_off[b];
    int lp = k.blklp[b];
    if (lp % n == 0) {
        if (k.defer_rot && n >= ROT_DEFER_MIN) {   // rot_kernel draws it and finishes this proposal
            k.pend_rot = b;
            return;
        }
        rot_matrix(k, off, n);
        lp = 0;
        if (n == 1) {   // a fresh one-parameter rotation every step: its sign is in hand
            k.blklp[b] = 1;
            proposal_r(c, t, k, b, 1, k.r1);
            return;
        }
    }
    proposal_tail(c, t, k, b, lp);
}

// ProposeVec after the rotation check: loop index, step length, UpdateParams
__device__ void proposal_tail(const DevCfg &c, const Tabs &t, Walker &k, int b, int lp)
{
    const int n = t.blk_n[b];
    const int off = t.blk_R_off[b];
    lp++;
    k.blklp[b] = lp;
    // vec(q) = R(q, loopix) (the column of R is read once: R may live in HBM
    // when it is too big to stage), scaled by Propose_r's step below
    for (int q0 = 0; !k.col_pre && q0 < n; q0 += RCH) {
        double rv[RCH];
#pragma unroll
        for (int u = 0; u < RCH; u++) rv[u] = q0 + u < n ? k.R[off + (q0 + u) * n + (lp - 1)] : 0.0;
#pragma unroll
        for (int u = 0; u < RCH; u++)
            if (q0 + u < n) k.vec[q0 + u] = rv[u];
    }
    proposal_r(c, t, k, b, n, 0.0);
}

// Propose_r's step length and UpdateParams: vec *= r * wid (r1: the 1 x 1
// rotation itself, when n == 1 and it was just drawn), P(changed) += mapping . vec
__device__ void proposal_r(const DevCfg &c, const Tabs &t, Walker &k, int b, int n, double r1)
{
    double rf;
    if (ranmar(k.r) < 0.33) {
        rf = (double)randexp1(k.r);
    } else {
        const int m = n < 2 ? n : 2;
        rf = 0.0;
        for (int i = 0; i < m; i++) {
            const double g = gaussian1(k.r);
            rf += g * g;
        }
        rf = sqrt(rf / m);
    }
    const double scale = rf * c.propose_scale;
    const int nc = t.blk_nchanged[b];
    const double *M = t.mapping + t.blk_map_off[b];
    const int *chg = t.changed + t.blk_changed_off[b];
    if (r1 != 0.0) k.vec[0] = r1 * scale;
    else
        for (int q0 = 0; q0 < n; q0 += RCH) {   // RCH loads in flight
            double v[RCH];
#pragma unroll
            for (int u = 0; u < RCH; u++) v[u] = k.vec[q0 + u < n ? q0 + u : 0];
#pragma unroll
            for (int u = 0; u < RCH; u++)
                if (q0 + u < n) k.vec[q0 + u] = v[u] * scale;
        }
    if (k.defer) {
        k.pend_b = b;
        return;
    }
    for (int j = 0; j < nc; j++) {
        double s = 0.0;
        for (int q = 0; q < n; q++) s += M[j * n + q] * k.vec[q];
        k.trial[chg[j]] += s;
    }
}

__device__ __forceinline__ void proposal_fast(const DevCfg &c, const Tabs &t, Walker &k)
{   // :283-289
    const int q = cyc_next(k, 2, c.fast_n, c.all_n + c.slow_n);
    block_proposal(c, t, k, t.pfi[c.slow_n + q - 1]);
}

__device__ __forceinline__ void proposal_slow(const DevCfg &c, const Tabs &t, Walker &k)
{   // :275-281
    const int q = cyc_next(k, 1, c.slow_n, c.all_n);
    block_proposal(c, t, k, t.pfi[q - 1]);
}

__device__ __forceinline__ void proposal(const DevCfg &c, const Tabs &t, Walker &k)
{   // GetProposal :257-273
    if (k.fast_ix != 0) {
        proposal_fast(c, t, k);
        k.fast_ix--;
    } else if (cyc_next(k, 0, c.all_n, 0) > c.slow_n) {
        proposal_fast(c, t, k);
        k.fast_ix = c.oversample_fast - 1;
    } else {
        proposal_slow(c, t, k);
    }
}

// GetLogLike calclike.f90:136-151 with AddLikeTemp :82-94; likes[l] are the
// data-likelihood terms at q (LogLikeWithTheorySet :374-387)
// test_row(i): row i of covinv . (q - center) (TestLikelihoodFunction's inner sum)
template <class Q>
__device__ inline double test_row(const DevCfg &c, const Tabs &t, const Q &q, int i)
{
    const int n = c.n_used;
    double s = 0.0;
    for (int j = 0; j < n; j++) s += t.covinv[i * n + j] * (q[t.params_used[j]] - t.center[t.params_used[j]]);
    return s;
}

// trows (stride MB), when given, holds (q - center)_i x test_row(i) for every
// i, computed by the other waves of mh_kernel: the same products, summed here
// in the same order (built with -ffp-contract=off: no fused multiply-add)
// zrows / oobv (stride MB), when given, hold every parameter's squared prior z
// (0 where there is no prior) and the bounds verdict of q, formed by the other
// thread groups: the same terms, summed here in the same order
template <class Q, class L>
__device__ __forceinline__ double target_like(const DevCfg &c, const Tabs &t, const Q &q, const L &likes,
                              const double *trows = nullptr, const double *zrows = nullptr, const int *oobv = nullptr)
{
    // the parameter loops load RCH entries at a time (all in flight together;
    // the chain wave would otherwise wait out one LDS round trip per entry)
    bool oob = oobv ? *oobv != 0 : false;
    for (int i0 = 0; !oobv && i0 < c.np; i0 += RCH) {                // GetLogLikeBounds :97-109
        double qv[RCH], hi[RCH], lo[RCH];
#pragma unroll
        for (int u = 0; u < RCH; u++) {
            const int i = i0 + u < c.np ? i0 + u : 0;
            qv[u] = q[i];
            hi[u] = t.pmax[i];
            lo[u] = t.pmin[i];
        }
#pragma unroll
        for (int u = 0; u < RCH; u++)
            if (i0 + u < c.np && (qv[u] > hi[u] || qv[u] < lo[u])) oob = true;
    }
    if (oob) return LOGZERO;
    double main = 0.0;
    if (c.test_like) {                                               // TestLikelihoodFunction :180-199
        const int n = c.n_used;
        double d = 0.0;
        for (int i0 = 0; trows && i0 < n; i0 += RCH) {   // the products, formed by the thread groups
            double v[RCH];
#pragma unroll
            for (int u = 0; u < RCH; u++) v[u] = trows[(size_t)(i0 + u < n ? i0 + u : 0) * MB];
#pragma unroll
            for (int u = 0; u < RCH; u++)
                if (i0 + u < n) d += v[u];
        }
        for (int i = 0; !trows && i < n; i++)
            d += (q[t.params_used[i]] - t.center[t.params_used[i]]) * test_row(c, t, q, i);
        main = d / 2.0;
    }
    for (int l = 0; l < c.n_like; l++) {
        const double v = likes[l];
        if (v == LOGZERO) return LOGZERO;
        main += v;
    }
    double like = main / c.temperature;
    if (c.has_priors) {                                              // GetLogPriors :111-134
        double pri = 0.0;
        for (int i0 = 0; zrows && i0 < c.np; i0 += RCH) {
            double zv[RCH];
#pragma unroll
            for (int u = 0; u < RCH; u++) zv[u] = zrows[(size_t)(i0 + u < c.np ? i0 + u : 0) * MB];
#pragma unroll
            for (int u = 0; u < RCH; u++)
                if (i0 + u < c.np) pri += zv[u];
        }
        for (int i0 = 0; !zrows && i0 < c.np; i0 += RCH) {   // std already 0 where the varying/include_fixed gate (:119) is off
            double qv[RCH], mu[RCH], sd[RCH];
#pragma unroll
            for (int u = 0; u < RCH; u++) {
                const int i = i0 + u < c.np ? i0 + u : 0;
                qv[u] = q[i];
                mu[u] = t.pmean[i];
                sd[u] = t.pstd[i];
            }
#pragma unroll
            for (int u = 0; u < RCH; u++)
                if (i0 + u < c.np && sd[u] != 0.0) {
                    const double z = (qv[u] - mu[u]) / sd[u];
                    pri += z * z;
                }
        }
        for (int k = 0; k < c.n_lin; k++)    // linear combinations :125-131
            if (t.lin_s[k] != 0.0) {
                const double *wk = t.lin_w + (size_t)k * c.np;
                double s = 0.0;
                for (int i = 0; i < c.np; i++) s += wk[i] * q[i];
                const double z = (s - t.lin_m[k]) / t.lin_s[k];
                pri += z * z;
            }
        like = like + (pri / 2.0) / c.temperature;
    }
    return like;
}

// Phase timestamps (s_memtime) of the first 64 mh_kernel blocks, only in the
// instrumented build (make EXTRA=-DCMAMD_STAMPS; tools/mh_stamps.py).
#ifdef CMAMD_STAMPS
__device__ unsigned long long g_stamps[64][16];
#define STAMP(i)                                                                                \
    do {                                                                                        \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                            \
        if (ACCEPT && PROPOSE && lane == 0 && wave == 0 && blockIdx.x < 64) g_stamps[blockIdx.x][i] = t_;            \
    } while (0)
#else
#define STAMP(i) ((void)0)
#endif

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;

// LDS-DMA (global_load_lds_dwordx4): rows [r0, r0+n) of a [rows][ld] double
// array, columns wb..wb+MB-1, into LDS rows [d0, d0+n) of [row][MB].  One wave
// instruction moves 1 KB (64 lanes x 16 bytes), i.e. 1024 / (8 MB) rows, and
// nothing passes through VGPRs, so every piece of the walker state is in
// flight at once.  Lanes past the last row are off.
__device__ inline void dma_rows_f64(double *dst, int d0, const double *src, int r0, int n, size_t ld, int wb,
                                    int lane, int wave = 0, int nw = 1)
{
    constexpr int LPR = MB / 2, RPI = 64 / LPR;   // lanes per row, rows per instruction
    for (int r = RPI * wave; r < n; r += RPI * nw) {
        const int rr = r + lane / LPR;
        if (rr < n) {
            const double *g = src + (size_t)(r0 + rr) * ld + wb + 2 * (lane % LPR);
            __builtin_amdgcn_global_load_lds((gbl_void_t *)g, (lds_void_t *)(dst + (size_t)(d0 + r) * MB), 16, 0, 0);
        }
    }
}

// same for int rows
__device__ inline void dma_rows_i32(int *dst, const int *src, int n, size_t ld, int wb, int lane, int wave = 0,
                                    int nw = 1)
{
    constexpr int LPR = MB / 4, RPI = 64 / LPR;
    for (int r = RPI * wave; r < n; r += RPI * nw) {
        const int rr = r + lane / LPR;
        if (rr < n) {
            const int *g = src + (size_t)rr * ld + wb + 4 * (lane % LPR);
            __builtin_amdgcn_global_load_lds((gbl_void_t *)g, (lds_void_t *)(dst + (size_t)r * MB), 16, 0, 0);
        }
    }
}

// flat copy of n 4-byte words (source allocation padded to a multiple of 64 words)
__device__ inline void dma_words(void *dst, const void *src, int n, int lane, int wave = 0, int nw = 1)
{
    for (int i = 64 * wave; i < n; i += 64 * nw) {
        const unsigned *g = reinterpret_cast<const unsigned *>(src) + i + lane;
        __builtin_amdgcn_global_load_lds((gbl_void_t *)g, (lds_void_t *)(reinterpret_cast<unsigned *>(dst) + i), 4,
                                         0, 0);
    }
}

// write-back of LDS rows [row][MB] (src rows src_r0 + (r - r0)) to HBM rows r
// in [r0, r1), columns wb .. wb+MB-1: 16 bytes per thread (MB = 16 doubles is 8
// threads a row, 16 ints 4 threads), all threads of the block, rows round-robin
template <class T>
__device__ inline void stage_out(T *dst, const T *src, int src_r0, int r0, int r1, size_t ld, int wb)
{
    constexpr int PER = 16 / sizeof(T), TPR = MB / PER, RPB = MH_THREADS / TPR;   // per thread, threads per row, rows per pass
    const int tr = threadIdx.x / TPR, col = (threadIdx.x % TPR) * PER;
    for (int r = r0 + tr; r < r1; r += RPB)
        *reinterpret_cast<uint4 *>(dst + (size_t)r * ld + wb + col) =
            *reinterpret_cast<const uint4 *>(src + (size_t)(src_r0 + r - r0) * MB + col);
}

// changeMask of the trial (TheoryLike_GetLogLikeMain, calclike.f90:302-306):
// likelihood l must be recomputed iff a parameter it depends on moved
// (LogLikeWithTheorySet :377); 1 = recompute, 0 = keep the current term
template <class QT, class QP>
__device__ inline void write_like_flags(const DevCfg &c, const QT &trial, const QP &P, int w)
{
    for (int l = 0; l < c.n_like; l++) {
        const unsigned long long m = c.like_dep[l];
        bool ch = false;
        for (int i = 0; i < c.np; i++)
            if (((m >> i) & 1ull) && trial[i] != P[i]) ch = true;
        c.like_flag[(size_t)l * c.ld + w] = ch ? 1 : 0;
    }
}

// One launch per Metropolis step boundary: accept/reject the pending trial
// (MetropolisAccept MCMC.f90:119-131 + MoveDone :166-190), then propose the
// next trial (GetProposal / GetProposalFast) and scatter its nuisance
// parameters for the likelihood kernels.  MB walkers per block.
// A Metropolis workgroup of the unified step launch waits here until its
// walker tile's quadratic-form and chi^2 workgroups have arrived (TailWait),
// then acquires their write-through outputs.  The producers are all earlier in
// the grid and wait on nothing, so the count arrives; the wait still gives up
// after TAIL_WAIT_SPINS polls and sets the status word, which the next step
// call reports as an error (sampler_check_pipe).  The bound counts polls, not
// wall-clock time: a poll does not advance while the wave is switched out (a
// shared GPU), so a waiter restored before its producers never gives up early.
// The per-tile arrival counters each on a line of their own (TW_PAD words
// apart), and the waiters poll them every TW_SLEEP x 64 cycles: the counters
// are agent-scope, so every poll and arrival goes past the XCD's L2, and 64
// waiters polling one line in a tight loop slow the quadratic form's own
// loads on the chip.
#ifndef CMAMD_TW_SLEEP
#define CMAMD_TW_SLEEP 20
#endif
#ifndef CMAMD_TW_PAD
#define CMAMD_TW_PAD 64
#endif
static constexpr int TW_PAD = CMAMD_TW_PAD;
// walkers per chi^2 workgroup in the unified launch (4 / 8 / 16: 35.7-35.8 /
// 35.9-36.0 / 35.9-36.0 us per middle launch, round 5)
#ifndef CMAMD_UNI_WT
#define CMAMD_UNI_WT 4
#endif
static constexpr int UNI_WT = CMAMD_UNI_WT;
// the pass role's weight prefetch: one step ahead (0), or two as the standalone
// kernels (1: measured 0.3 us slower a launch with 288-l items, and the same
// within noise with 352-l items: 32.6 / 32.0 / 31.8 against 32.1 / 32.4 / 31.9 us, round 6)
#ifndef CMAMD_UNI_W2
#define CMAMD_UNI_W2 0
#endif
static constexpr long TAIL_WAIT_SPINS = (1l << 25) / CMAMD_TW_SLEEP;   // polls: ~1 s

// A give-up: the sampler's status word lives in pinned host memory (mapped),
// so the host reads it once the step call's event has completed, without a
// copy launch; every writer stores the same bit, so a plain system-scope store
// serves (no read-modify-write over the bus)
__device__ __forceinline__ void pipe_giveup(int *status)
{
    __hip_atomic_store(status, CMBL_STATUS_PIPE_WAIT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void tail_wait(const TailWait &tw, int tile)
{
    if (threadIdx.x == 0) {
        const int gpt = 64 / tw.gwt, g0 = tile * gpt;
        const int gq = max(0, min(gpt, tw.ng - g0));
        // every accepting launch adds its quadratic-form workgroups, and those whose
        // chi^2 ran as workgroups of its own (not folded) add the tile's chi^2 ones
        const unsigned target = tw.epoch * (unsigned)tw.nq_items + tw.epoch_g * (unsigned)gq;
        for (long it = 0;; it++) {
            const unsigned v = __hip_atomic_load(tw.cnt + tile * TW_PAD, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (v >= target) break;
            if (it == TAIL_WAIT_SPINS) {
                pipe_giveup(tw.status);
                break;
            }
            __builtin_amdgcn_s_sleep(CMAMD_TW_SLEEP);
        }
        // one acquire after the match (cdna_hip_programming.md Guideline 16 recipe): it drops this
        // CU's L1 lines; its own wait holds the barrier, then every wave loads
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifdef CMAMD_STAMPS
        if (blockIdx.x < 2048) g_uni_stamps[tw.stamp_slot][blockIdx.x][1] = __builtin_amdgcn_s_memrealtime();
#endif
    }
    __syncthreads();
}

#include "mhlean.h"

// tw: the unified step launch's wait (mh_step_kernel), else null
template <bool ACCEPT, bool PROPOSE>
__device__ __forceinline__ void mh_body(const DevCfg &c, int fast_only, double *hist_row, double *hist_terms, int blk0,
                                        double *lds, int bx, const TailWait *tw = nullptr)
{
    if (c.lean.on) {   // a single one-parameter fast block (mhlean.h)
        mh_lean<ACCEPT, PROPOSE>(c, hist_row, hist_terms, blk0, lds, bx, tw);
        return;
    }
    const Rows &R = c.rows;
    const int lane = threadIdx.x % MB, grp = threadIdx.x / MB;    // walker in block, thread group
    const int wl64 = threadIdx.x & 63, wave = threadIdx.x >> 6, nwave = MH_THREADS / 64;
    const int wb = (blk0 + bx) * MB;
    const int w = wb + lane;
    const bool act = w < c.W;
    const size_t W = c.ld;
    const int nlk = (c.n_like + 1) & ~1;
    // LDS carve: state doubles | like terms | vec scratch | tables(d) | state ints | itmp | tables(i)
    const int nd_st = c.stage_R ? R.ND : R.ND - R.RR;           // staged double rows
    const int ni_st = c.stage_cyc ? R.NI : R.CYC;                // staged int rows
    const int ntd = c.stage_cov ? c.tl.n_dbl : c.tl.covinv;      // staged double-table words
    double *sd = lds;                                            // [nd_st][MB]
    double *lk = sd + (size_t)nd_st * MB;                        // [nlk][MB]
    double *vc = lk + (size_t)nlk * MB;                          // [max_blk][MB]
    double *tq = vc + (size_t)c.max_blk * MB;                    // [tq_rows][MB] test-Gaussian row sums / block
    double *dq = tq + (size_t)c.tq_rows * MB;                    // [def_cap][QF_GROUPS + 1][MB] deferred combines
    double *td = dq + (size_t)c.def_cap * (QF_GROUPS + 1) * MB;  // [ntd rounded to 32]
    int *si = reinterpret_cast<int *>(td + ((ntd + 31) & ~31));  // [ni_st][MB]
    int *it = si + (size_t)ni_st * MB;                           // [all_n][MB] when stage_cyc
    int *ti = it + (size_t)(c.stage_cyc ? c.all_n : 0) * MB;     // [n_int rounded to 64]
    int *oobw = ti + ((c.tl.n_int + 63) & ~63);                  // [MB] trial out of bounds (par_prior)
    double *zz = reinterpret_cast<double *>(oobw + MB);          // [np][MB] the trial's squared prior z (par_prior)
    int *ndw = reinterpret_cast<int *>(zz + (size_t)c.np * MB);  // [MB] ring entries the chain's draws wrote
    int *i0w = ndw + MB;                                         // [MB] the ring index before them
    if (threadIdx.x < MB) oobw[threadIdx.x] = 0;
    // the rotation list of this walker range: this launch appends to counter
    // rot_par; the other one (read by the previous step's rot_kernel) restarts
    if (PROPOSE && c.rot_defer && bx == 0 && threadIdx.x == 0)
        c.rot_cnt[2 * (blk0 * MB / 64) + (c.rot_par ^ 1)] = 0;
    const bool skipR = !c.stage_R;
    // staged double row index of global row r (rotation rows dropped when not staged)
#define SROW(r) ((skipR && (r) >= R.R) ? (r) - R.RR : (r))

    STAMP(0);
    // every wave issues the LDS-DMA of the state image; lanes 0..MB-1 of wave
    // 0 alone run the chain logic; every thread group writes the image back
    const int rEnd = R.R + R.RR;
    if (skipR) {
        dma_rows_f64(sd, 0, c.sd, 0, R.R, W, wb, wl64, wave, nwave);
        dma_rows_f64(sd, R.R, c.sd, rEnd, R.ND - rEnd, W, wb, wl64, wave, nwave);
    } else {
        dma_rows_f64(sd, 0, c.sd, 0, R.ND, W, wb, wl64, wave, nwave);
    }
    dma_rows_i32(si, c.si, ni_st, W, wb, wl64, wave, nwave);
    dma_words(td, c.tab_d, 2 * ntd, wl64, wave, nwave);
    dma_words(ti, c.tab_i, c.tl.n_int, wl64, wave, nwave);
    // fast-only proposals with R in HBM: the only fast block's next column
    // (R(:, lp + 1) when no rotation is due) fetched into the vec rows by the
    // thread groups (proposal_tail then skips its own read; a block that
    // rotates writes R only in rot_kernel).  When the host knows the loop
    // index (pre_lp) the loads go out here, beside the image; otherwise after
    // it, from the staged index
    const bool pre_col = PROPOSE && fast_only && !c.stage_R && c.pre_blk >= 0;
    constexpr int NRQ = (MAXBLK + NV - 1) / NV;
    double rq[NRQ];
    int col = -1, ncol = 0;
    const bool rq_early = pre_col && c.pre_lp >= 0;
    if (rq_early && act) {
        ncol = c.pre_n;
        if (c.pre_lp % ncol != 0) col = c.pre_off + c.pre_lp;
#pragma unroll
        for (int u = 0; u < NRQ; u++) {
            const int q = grp + u * NV;
            if (col >= 0 && q < ncol) rq[u] = c.sd[(size_t)(R.R + col + q * ncol) * W + w];
        }
    }
    if (tw) tail_wait(*tw, wb / 64);   // the trial's terms below come from this launch's producers
    dma_rows_f64(lk, 0, c.like_terms, 0, nlk, W, wb, wl64, wave, nwave);
    // per-likelihood terms of the current point, for the history (rejected walkers keep theirs)
    double ct[MAXLIKE];
    if (ACCEPT && hist_terms && grp == 0 && act) {
#pragma unroll
        for (int l = 0; l < MAXLIKE; l++)
            if (l < c.n_like) ct[l] = c.cur_terms[(size_t)l * W + w];
    }
    // deferred split-K combines: the 16 group sums of this walker tile's
    // partials, one group per wave, loaded beside the state image
    if (ACCEPT && c.n_def) {   // group g sums split-K group g of this block's walkers (columns wb % 64 + lane of the tile)
        const int tile = wb / QF_TILE, col = wb % QF_TILE + lane;
        for (int d = 0; d < MAXDEF; d++) {
            if (d >= c.n_def) break;
            const double *tp = c.def_part[d] + (size_t)tile * c.def_items[d] * QF_TILE;
            double *row = dq + (size_t)d * (QF_GROUPS + 1) * MB;
            if (grp < QF_GROUPS) row[(size_t)grp * MB + lane] = qf_group_sum(tp, c.def_items[d], grp, col);
            if (grp == NV - 1) row[(size_t)QF_GROUPS * MB + lane] = (c.def_add[d] && act) ? c.def_add[d][w] : 0.0;
        }
    }
    STAMP(1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (ACCEPT && c.n_def && grp == 0 && act) {   // finish them in quadform.h's fixed order
        for (int d = 0; d < MAXDEF; d++) {
            if (d >= c.n_def) break;
            const double *row = dq + (size_t)d * (QF_GROUPS + 1) * MB;
            double v = qf_tree(row + lane, MB);
            if (c.def_add[d]) v = v + row[(size_t)QF_GROUPS * MB + lane];
            const int l = c.def_like[d];
            lk[(size_t)l * MB + lane] = v;
            const_cast<double *>(c.like_terms)[(size_t)l * W + w] = v;
        }
    }
    // the test-Gaussian rows of covinv . (trial - center) are spread over the
    // waves (each row summed by one thread, in order) instead of run serially
    // by the chain wave: first the differences (trial - center)_j, one row
    // each (tq rows n_used ..), then the rows' sums and their products with
    // the differences (tq rows 0 ..), every sum's loads in flight together
    const bool par_test = ACCEPT && c.test_like && c.n_used >= 4 && c.tq_rows >= 2 * c.n_used;
    const bool par_map = PROPOSE && c.max_blk >= 4 && c.tq_rows >= 2;
    // the trial's bounds check and squared Gaussian-prior z of every parameter,
    // spread over the thread groups (the chain thread then only sums them in order)
    const bool par_prior = ACCEPT;
    if (par_test || par_prior || pre_col) {
        if (pre_col && !rq_early && act) {
            const int b = c.pre_blk, off = ti[c.tl.blk_R_off + b];
            ncol = ti[c.tl.blk_n + b];
            const int lp = si[(size_t)(R.BLKLP + b) * MB + lane];
            if (lp % ncol != 0) col = off + lp;
#pragma unroll
            for (int u = 0; u < NRQ; u++) {
                const int q = grp + u * NV;
                if (col >= 0 && q < ncol) rq[u] = c.sd[(size_t)(R.R + col + q * ncol) * W + w];
            }
        }
        const Tabs t0 = make_tabs(c, ti, td, c.stage_cov ? td : c.tab_d);
        const Col<double> q{sd + (size_t)SROW(R.T) * MB + lane, MB};
        const int nu = c.n_used;
        double *dif = tq + (size_t)nu * MB + lane;
        if (act) {
            if (par_test)
                for (int i = grp; i < nu; i += NV) {
                    const int pi = t0.params_used[i];
                    dif[(size_t)i * MB] = q[pi] - t0.center[pi];
                }
            if (par_prior) {
                int oob = 0;
                for (int i = grp; i < c.np; i += NV) {
                    const double qv = q[i];
                    if (qv > t0.pmax[i] || qv < t0.pmin[i]) oob = 1;   // GetLogLikeBounds :97-109
                    double z2 = 0.0;
                    if (c.has_priors && t0.pstd[i] != 0.0) {           // GetLogPriors :111-124
                        const double z = (qv - t0.pmean[i]) / t0.pstd[i];
                        z2 = z * z;
                    }
                    zz[(size_t)i * MB + lane] = z2;
                }
                if (oob) atomicOr(&oobw[lane], 1);
            }
        }
        if (par_test) {
            __syncthreads();
            if (act)
                for (int i = grp; i < nu; i += NV) {   // test_row's sum, same order
                    const double *ci = t0.covinv + (size_t)i * nu;
                    double s = 0.0;
                    for (int j0 = 0; j0 < nu; j0 += RCH) {
                        double cv[RCH], dv[RCH];
#pragma unroll
                        for (int u = 0; u < RCH; u++) {
                            const int j = j0 + u < nu ? j0 + u : 0;
                            cv[u] = ci[j];
                            dv[u] = dif[(size_t)j * MB];
                        }
#pragma unroll
                        for (int u = 0; u < RCH; u++)
                            if (j0 + u < nu) s += cv[u] * dv[u];
                    }
                    tq[(size_t)i * MB + lane] = dif[(size_t)i * MB] * s;
                }
        }
#pragma unroll
        for (int u = 0; u < NRQ; u++) {
            const int qq = grp + u * NV;
            if (col >= 0 && qq < ncol) vc[(size_t)qq * MB + lane] = rq[u];
        }
        __syncthreads();
    }
    STAMP(2);
    if (grp == 0 && act) {

    const Tabs t = make_tabs(c, ti, td, c.stage_cov ? td : c.tab_d);
    Walker k;
    k.r.u = Col<double>{sd + (size_t)R.U * MB + lane, MB};
    k.r.c = sd[(size_t)R.C * MB + lane];
    k.r.gset = sd[(size_t)R.G * MB + lane];
    k.r.i97 = si[(size_t)R.I97 * MB + lane];
    k.r.j97 = si[(size_t)R.J97 * MB + lane];
    k.r.iset = si[(size_t)R.ISET * MB + lane];
    k.R = c.stage_R ? Col<double>{sd + (size_t)R.R * MB + lane, MB} : Col<double>{c.sd + (size_t)R.R * W + w, c.ld};
    k.P = Col<double>{sd + (size_t)SROW(R.P) * MB + lane, MB};
    k.trial = Col<double>{sd + (size_t)SROW(R.T) * MB + lane, MB};
    k.vec = Col<double>{vc + lane, MB};
    k.cyc = c.stage_cyc ? Col<int>{si + (size_t)R.CYC * MB + lane, MB} : Col<int>{c.si + (size_t)R.CYC * W + w, c.ld};
    k.cyclp = Col<int>{si + (size_t)R.CYCLP * MB + lane, MB};
    k.blklp = Col<int>{si + (size_t)R.BLKLP * MB + lane, MB};
    k.itmp = c.stage_cyc ? Col<int>{it + lane, MB} : Col<int>{c.itmp_g + w, c.ld};
    k.fast_ix = si[(size_t)R.FASTIX * MB + lane];
    const int i97_0 = k.r.i97;
    double &cur = sd[(size_t)SROW(R.L) * MB + lane];
    double &mult = sd[(size_t)SROW(R.M) * MB + lane];
    int &nacc = si[(size_t)R.NACC * MB + lane];

    bool moved = false;   // accepted: P = trial already
    if (ACCEPT) {
        if (c.mask_on) {   // unchanged likelihoods keep the current point's term (calclike.f90:377-384)
            for (int l = 0; l < c.n_like; l++) {
                const int f = c.like_flag[(size_t)l * W + w];
                double v;
                if (f == 0) v = c.cur_terms[(size_t)l * W + w];
                else if (c.like_out[l]) v = c.like_out[l][f - 1];        // sparse: compacted slot
                else v = lk[(size_t)l * MB + lane];
                lk[(size_t)l * MB + lane] = v;
            }
        }
        STAMP(8);
        const double like = target_like(c, t, k.trial, Col<double>{lk + lane, MB}, par_test ? tq + lane : nullptr,
                                        par_prior ? zz + lane : nullptr, par_prior ? oobw + lane : nullptr);
        STAMP(9);
        bool acc = false;
        if (like != LOGZERO) {
            acc = cur > like;
            if (!acc) acc = (double)randexp1(k.r) > like - cur;
        }
        STAMP(10);
        moved = acc;
        if (acc) {
            if (mult > 0) nacc += 1;
            mult = 1.0;
            for (int i0 = 0; !par_map && i0 < c.np; i0 += RCH) {   // P = trial (par_map: the groups, below)
                double v[RCH];
#pragma unroll
                for (int u = 0; u < RCH; u++) v[u] = k.trial[i0 + u < c.np ? i0 + u : 0];
#pragma unroll
                for (int u = 0; u < RCH; u++)
                    if (i0 + u < c.np) k.P[i0 + u] = v[u];
            }
            cur = like;
#pragma unroll
            for (int l = 0; l < MAXLIKE; l++)
                if (l < c.n_like) {
                    ct[l] = lk[(size_t)l * MB + lane];
                    c.cur_terms[(size_t)l * W + w] = ct[l];
                }
        } else {
            mult += 1.0;
        }
        STAMP(11);
        si[(size_t)R.ACCF * MB + lane] = acc ? 1 : 0;
        if (par_map) oobw[lane] = acc ? 1 : 0;   // (target_like has read the bounds verdict)
        if (hist_row) hist_row[(size_t)c.n_used * c.W + w] = cur;   // the parameters: every group, below
        if (hist_terms) {
#pragma unroll
            for (int l = 0; l < MAXLIKE; l++)
                if (l < c.n_like) hist_terms[(size_t)l * c.W + w] = ct[l];
        }
    }
    STAMP(3);
    if (PROPOSE) {
        for (int i0 = 0; !moved && !par_map && i0 < c.np; i0 += RCH) {   // Trial = CurParams (par_map: below)
            double v[RCH];
#pragma unroll
            for (int u = 0; u < RCH; u++) v[u] = k.P[i0 + u < c.np ? i0 + u : 0];
#pragma unroll
            for (int u = 0; u < RCH; u++)
                if (i0 + u < c.np) k.trial[i0 + u] = v[u];
        }
        STAMP(14);
        k.defer = par_map;
        k.defer_rot = c.rot_defer;
        k.col_pre = pre_col && k.blklp[c.pre_blk] % t.blk_n[c.pre_blk] != 0 &&
                    (!rq_early || k.blklp[c.pre_blk] == c.pre_lp);   // else proposal_tail reads the column itself
        if (fast_only) proposal_fast(c, t, k);
        else proposal(c, t, k);
        STAMP(15);
        si[(size_t)R.PROT * MB + lane] = k.pend_rot + 1;             // rot_kernel finishes this walker
        if (k.pend_rot >= 0) {
            const int slot = atomicAdd(c.rot_cnt + 2 * (blk0 * MB / 64) + c.rot_par, 1);
            c.rot_list[blk0 * MB + slot] = w;
            if (par_map) tq[lane] = -1.0;
        } else if (par_map) tq[lane] = (double)k.pend_b;             // the block, for the mapping waves
        else {
            for (int l = 0; l < c.n_like; l++)
                for (int q = 0; q < c.like_nn[l]; q++)
                    c.like_nuis[l][(size_t)w * c.like_nn[l] + q] = k.trial[t.ti[c.like_nidx[l] + q]];
            if (c.mask_on) write_like_flags(c, k.trial, k.P, w);
        }
    }
    STAMP(4);
    sd[(size_t)R.C * MB + lane] = k.r.c;
    sd[(size_t)R.G * MB + lane] = k.r.gset;
    si[(size_t)R.I97 * MB + lane] = k.r.i97;
    si[(size_t)R.J97 * MB + lane] = k.r.j97;
    si[(size_t)R.ISET * MB + lane] = k.r.iset;
    si[(size_t)R.FASTIX * MB + lane] = k.fast_ix;
    ndw[lane] = k.r.nd < 97 ? k.r.nd : 97;
    i0w[lane] = i97_0;
    }
    if (par_map) {   // UpdateParams' mapping product, rows spread over the waves (one thread per row, same order)
        __syncthreads();
        // first P = trial (accepted) or trial = P (rejected, or no accept in
        // this launch: oobw is 0), the chain having left both to the groups
        if (act) {
            double *Pr = sd + (size_t)SROW(R.P) * MB + lane, *Tr = sd + (size_t)SROW(R.T) * MB + lane;
            const bool mv = oobw[lane] != 0;
            for (int i = grp; i < c.np; i += NV) {
                if (mv) Pr[(size_t)i * MB] = Tr[(size_t)i * MB];
                else Tr[(size_t)i * MB] = Pr[(size_t)i * MB];
            }
        }
        __syncthreads();
        if (act && tq[lane] >= 0.0) {
            const Tabs t = make_tabs(c, ti, td, c.stage_cov ? td : c.tab_d);
            const int b = (int)tq[lane];
            const int n = t.blk_n[b], nc = t.blk_nchanged[b];
            const double *M = t.mapping + t.blk_map_off[b];
            const int *chg = t.changed + t.blk_changed_off[b];
            double *trial = sd + (size_t)SROW(R.T) * MB + lane;
            const double *vec = vc + lane;
            for (int j = grp; j < nc; j += NV) {
                double s = 0.0;
#pragma unroll 4
                for (int q = 0; q < n; q++) s += M[j * n + q] * vec[(size_t)q * MB];
                trial[(size_t)chg[j] * MB] += s;
            }
        }
        __syncthreads();
        STAMP(12);
        if (grp == 0 && act && si[(size_t)R.PROT * MB + lane] == 0) {
            const double *trial = sd + (size_t)SROW(R.T) * MB + lane;
            for (int l = 0; l < c.n_like; l++)
                for (int q = 0; q < c.like_nn[l]; q++)
                    c.like_nuis[l][(size_t)w * c.like_nn[l] + q] = trial[(size_t)ti[c.like_nidx[l] + q] * MB];
            if (c.mask_on)
                write_like_flags(c, Col<const double>{trial, MB}, Col<const double>{sd + (size_t)SROW(R.P) * MB + lane, MB},
                                 w);
        }
    }
    __syncthreads();
    STAMP(13);
    if (ACCEPT && hist_row && act) {   // the history row's parameters (P is final), rows spread over the groups
        const int *pu = ti + c.tl.params_used;
        for (int i = grp; i < c.n_used; i += NV)
            hist_row[(size_t)i * c.W + w] = sd[(size_t)(SROW(R.P) + pu[i]) * MB + lane];
    }
    if (PROPOSE && c.pub_on && threadIdx.x < MB && act)   // the fused pass / bins in this launch poll for these
        for (int k = 0; k < 2; k++) {
            const int pc = c.pub_pcal[k];
            const bool rp = si[(size_t)R.PROT * MB + lane] != 0;   // rot_kernel proposes it (bin co-run only)
            const double v = rp ? __longlong_as_double((long long)TP_PIPE_ROT)
                                : pc >= 0 ? sd[(size_t)(SROW(R.T) + pc) * MB + lane] : 1.0;
            __hip_atomic_store(c.calbuf + (size_t)k * W + w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(c.calbuf_next + (size_t)k * W + w, __longlong_as_double((long long)TP_PIPE_UNSET),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // read by the next launch only
        }
    // write back the image (rows of walkers past W are padding of the ld-wide
    // rows: written back unchanged) -- of the RANMAR ring only the entries
    // this launch's draws overwrote (positions i97 - 1, i97 - 2, ... mod 97
    // of the first index)
    if (act) {
        const int nd = ndw[lane], i0 = i0w[lane];
        for (int t = grp; t < nd; t += NV) {
            int p = i0 - 1 - t;
            if (p < 0) p += 97;
            c.sd[(size_t)(R.U + p) * W + w] = sd[(size_t)(R.U + p) * MB + lane];
        }
    }
    if (skipR) {
        stage_out(c.sd, sd, R.C, R.C, R.R, W, wb);
        stage_out(c.sd, sd, R.R, rEnd, R.ND, W, wb);
    } else {
        stage_out(c.sd, sd, R.C, R.C, R.ND, W, wb);
    }
    stage_out(c.si, si, 0, 0, ni_st, W, wb);
    STAMP(5);
#ifdef CMAMD_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    STAMP(6);
#endif
#undef SROW
}

template <bool ACCEPT, bool PROPOSE>
__global__ __launch_bounds__(MH_THREADS) void mh_kernel(DevCfg c, int fast_only, double *hist_row, double *hist_terms, int blk0)
{
    extern __shared__ __attribute__((aligned(16))) double lds[];
    mh_body<ACCEPT, PROPOSE>(c, fast_only, hist_row, hist_terms, blk0, lds, blockIdx.x);
}

// A proposing mh_kernel with plik_lite's binning riding along (the bin
// co-run of sampler_step): workgroups [0, nmh) are mh_kernel's, the pad up to
// a multiple of 8 idle, the rest bin a walker each (its three fields in
// turn: one workgroup per walker keeps the whole grid resident beside the
// Metropolis workgroups' LDS size; plik_bin_products and the bin sums), wait
// for the walker's trial calibration (published by its Metropolis workgroup
// into DevCfg::calbuf straight after the proposal) and emit
// Delta = X - S / cal^2 into plik's rows -- or, for a walker whose proposal
// waits on a new rotation (TP_PIPE_ROT), the raw sums, from which rot_kernel
// forms its Delta after the launch.  The binning runs on the CUs the
// latency-bound Metropolis chain leaves idle (it takes 32 of 256 at
// W = 512); only its emit waits.
// The bins wait on workgroups with lower ids.  The HIP model does not promise
// that workgroups are dispatched in id order (cdna_hip_programming.md
// "Workgroups, grid, and XCD partitioning"); the hardware's dispatcher is
// observed to, so the Metropolis workgroups are resident before any waiting
// bin workgroup takes a slot and the wait ends.  The design does not rely on
// it for correctness: the wait is bounded by a count of polls
// (TAIL_WAIT_SPINS), and a give-up sets CMBL_STATUS_PIPE_WAIT in the
// sampler's status word, which the next step call or state readback turns
// into an error (sampler_check_pipe) instead of silently rejected trials.
template <bool ACCEPT>
__global__ __launch_bounds__(MH_THREADS) void mh_bin_kernel(DevCfg c, int fast_only, double *hist_row,
                                                            double *hist_terms, int nmh, int nmh_pad, PlikBinArgs pb,
                                                            int *status)
{
    extern __shared__ __attribute__((aligned(16))) double lds[];
    __shared__ double cal_s;
    const int b = blockIdx.x;
    if (b < nmh_pad) {
        if (b < nmh) mh_body<ACCEPT, true>(c, fast_only, hist_row, hist_terms, 0, lds, b);
        return;
    }
    const int w = b - nmh_pad;
    for (int i = pb.nused + (int)threadIdx.x; i < pb.Np; i += MH_THREADS)   // the Delta row's padding columns
        c.bin_delta[(size_t)w * pb.Np + i] = 0.0;
    // the three fields in turn through one LDS image: this thread's bin sums
    // (plik_bin_emit's, at most two bins a field: bin_setup) before the wait,
    // so only the emit follows the calibration
    double acc[3][2] = {};
#pragma unroll
    for (int f = 0; f < 3; f++) {
        if (f > 0) __syncthreads();   // the previous field's sums have read the image
        if (!plik_bin_products(pb, lds, w, f)) continue;
        const double *P = lds - pb.fr.lo[f];
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const int i = pb.fr.b0[f] + (int)threadIdx.x + k * MH_THREADS;
            if (i < pb.fr.b1[f]) {
                const BinInfo bi = pb.bins[i];
                for (int l = bi.lmin; l <= bi.lmax; l++) acc[f][k] += P[l];
            }
        }
    }
    if (threadIdx.x == 0) {
        double cl;
        for (long it = 0;; it++) {   // bounded by polls (tail_wait): a safety net, reported loudly
            cl = __hip_atomic_load(c.calbuf + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((unsigned long long)__double_as_longlong(cl) != TP_PIPE_UNSET) break;
            if (it == (1l << 20)) {   // x s_sleep(24): ~0.7 s
                pipe_giveup(status);
                break;
            }
            __builtin_amdgcn_s_sleep(24);   // ~1500 cycles: 3 W pollers must not crowd the L2
        }
        cal_s = cl;
    }
    __syncthreads();
    const double cl = cal_s, c2 = cl * cl;
    const bool rot = (unsigned long long)__double_as_longlong(cl) == TP_PIPE_ROT;
    double *out = (rot ? const_cast<double *>(c.bin_S) : c.bin_delta) + (size_t)w * pb.Np;
#pragma unroll
    for (int f = 0; f < 3; f++)
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const int i = pb.fr.b0[f] + (int)threadIdx.x + k * MH_THREADS;
            if (pb.fr.hi[f] >= pb.fr.lo[f] && i < pb.fr.b1[f]) out[i] = rot ? acc[f][k] : pb.X[i] - acc[f][k] / c2;
        }
}

// The unified step launch (pipe_mode 3): one launch per fast step.  Rows of
// workgroups (tail_rows) run step k's tails -- plik_lite's quadratic form from
// raw sums and the lensing chi^2, which store write-through and arrive on
// their walker tile's counter -- the window pass storing step k + 1's raw sums,
// and last the Metropolis workgroups, which wait for their tile's arrivals
// (tail_wait), accept step k (finishing plik's deferred combine from the
// partials of this launch) and propose step k + 1.  The pass waits on
// nothing; the Metropolis chain of a tile starts as soon as its tails are
// done instead of at a kernel boundary, and overlaps the pass.
// The hand-off is cdna_hip_programming.md's counter recipe in its
// write-through form (the note to its split-K combine, after Guideline 16):
// the producers' stores are sc1 (write-through past the XCD L2), so no
// release fence precedes the relaxed agent-scope fetch_add -- every wave
// drains its stores, the workgroup barriers, one lane adds; the consumer
// polls relaxed and takes one acquire fence after the match (tail_wait).
// A release fence here would be a whole-L2 write-back per producer
// workgroup (measured on the pass units: 35.8 -> 122 us a launch).
__device__ __forceinline__ void tail_arrive(const TailWait &tw, int tile)
{
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's write-through stores are done
    __syncthreads();
    if (threadIdx.x == 0 && !tw.nosignal)
        __hip_atomic_fetch_add(tw.cnt + tile * TW_PAD, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool ACCEPT, bool PROPOSE>
__device__ __forceinline__ void mh_step_body(DevCfg &c, int fast_only, double *hist_row, double *hist_terms,
                                             StepTail &t, const int2 *__restrict__ rows, TailWait &tw, int nmh)
{
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int2 rr = rows[blockIdx.x >> 3];
    const int lb = rr.y * 8 + (blockIdx.x & 7);
    if (!ACCEPT && blockIdx.x == 0)   // a call's first launch (no tails): the arrival counters start from 0
        for (int i = threadIdx.x; i < tw.ntiles; i += MH_THREADS) tw.cnt[i] = 0u;
#ifdef CMAMD_STAMPS
    const bool stamp = ACCEPT && threadIdx.x == 0 && blockIdx.x < 2048;
    const int slot = PROPOSE ? 0 : 1;
    if (stamp) {
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        g_uni_stamps[slot][blockIdx.x][0] = __builtin_amdgcn_s_memrealtime();
        g_uni_stamps[slot][blockIdx.x][2] = xcc & 15;
        g_uni_stamps[slot][blockIdx.x][4] = 0;
        g_uni_stamps[slot][blockIdx.x][5] = 0;
    }
    struct End {
        bool on;
        int role, slot;
        __device__ ~End() {
            if (on) {
                g_uni_stamps[slot][blockIdx.x][3] = __builtin_amdgcn_s_memrealtime();
                g_uni_stamps[slot][blockIdx.x][4] = role + 1;
            }
        }
    } end_{stamp, rr.x, slot};
#endif
    if (rr.x == TAIL_QF) {
        if (lb >= t.nq) return;
        int item_ix, tile;
        qf_place(lb, t.q.src.n_items, t.q.src.xcd_map, item_ix, tile);
        // the quadratic form's waves above the pass's at issue (the Metropolis
        // waves' 3 stays highest): 35.98 / 36.26 -> 35.90 / 35.80 us per step in two
        // interleaved repetitions (round 6, tools/gpu_r6f.sh); CMAMD_QF_PRIO=0 turns it off
        if (t.qf_prio) __builtin_amdgcn_s_setprio(2);
        if (PROPOSE && t.qf_ahead)   // A/B (CMAMD_QF_AHEAD): the two-step-ahead form in the middle launches too
            qfs_body<true, true>(lds, item_ix, tile, t.q);
        else
            qfs_body<true, !PROPOSE>(lds, item_ix, tile, t.q);
        tail_arrive(tw, tile);
    } else if (rr.x == TAIL_GAUSS) {
        // contiguous walker groups per XCD (lb % 8 is the XCD): each partial row's
        // 128-byte lines are read by one XCD's L2 instead of four (35.1 -> 34.5 us)
        const int grows = (t.ng + 7) >> 3, q = (lb & 7) * grows + (lb >> 3);
        if (q >= t.ng) return;
        small_gauss_body<UNI_WT, true, true>(t.g, lds, q);
        tail_arrive(tw, q * UNI_WT / 64);
    } else if (rr.x == TAIL_PASS) {
        if (lb >= t.np) return;
        tp_vec_body<2, true, CMAMD_UNI_W2 != 0>(t.tp, t.dl, t.ld_field, t.ld_walker, t.W, reinterpret_cast<char *>(lds), lb);
    } else if (lb < nmh) {
        // the chain is latency on one lane: its waves, dispatched last (the youngest,
        // so the last in issue arbitration), take the SIMD first (34.6 -> 34.0 us)
        if (!t.fold_late_prio) __builtin_amdgcn_s_setprio(3);
        if (ACCEPT && t.fold_g) {
            // the small chi^2 of this workgroup's 16 walkers (step k's raw partial
            // rows, whole 128-byte lines) while the quadratic form runs elsewhere:
            // nX <= 16, so its sums are those of the 4-walker rows (same bits); the
            // chain's loads of the term follow tail_wait's acquire
            if (t.fold_tpf == 2) small_gauss_body<MB, true, false, 2>(t.g, lds, lb);
            else small_gauss_body<MB, true, false, 1>(t.g, lds, lb);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
#ifdef CMAMD_STAMPS
            if (threadIdx.x == 0 && blockIdx.x < 2048)
                g_uni_stamps[PROPOSE ? 0 : 1][blockIdx.x][5] = __builtin_amdgcn_s_memrealtime();
#endif
        }
        if (t.fold_late_prio) __builtin_amdgcn_s_setprio(3);   // A/B: the folded chi^2 at the default priority
        mh_body<ACCEPT, PROPOSE>(c, fast_only, hist_row, hist_terms, 0, lds, lb, ACCEPT ? &tw : nullptr);
    }
}

template <bool ACCEPT, bool PROPOSE>
__global__ __launch_bounds__(MH_THREADS, 3) void mh_step_kernel(DevCfg c, int fast_only, double *hist_row,
                                                                double *hist_terms, StepTail t,
                                                                const int2 *__restrict__ rows, TailWait tw, int nmh)
{
    mh_step_body<ACCEPT, PROPOSE>(c, fast_only, hist_row, hist_terms, t, rows, tw, nmh);
}

// The same launch without the pass, for the binned-theory cache
// (cmbs_set_binned_cache): its own symbol, so profiles of a run with both
// legs keep the headline launch's statistics apart
template <bool ACCEPT, bool PROPOSE>
__global__ __launch_bounds__(MH_THREADS, 3) void mh_tail_kernel(DevCfg c, int fast_only, double *hist_row,
                                                                double *hist_terms, StepTail t,
                                                                const int2 *__restrict__ rows, TailWait tw, int nmh)
{
    mh_step_body<ACCEPT, PROPOSE>(c, fast_only, hist_row, hist_terms, t, rows, tw, nmh);
}

// ------------------------------------------------------- deferred rotations
// A new random rotation of a block of ROT_DEFER_MIN or more parameters
// (RotMatrix propose.f90:88-102 -> RandRotationD RandUtils.f90:133-153) is too
// big for the chain lane: mh_kernel stops that walker's proposal at the
// rotation (Rows::PROT), appends the walker to the step's rotation list, and
// rot_kernel, one wave per listed walker, finishes it.
//
// The Gaussians.  RANMAR's lagged-Fibonacci part is x_m = x_{m-97} - x_{m-33}
// mod 1 (RandUtils.f90:350-374), an integer recurrence mod 2^24 in units of
// 2^-24, and its carry c_m = c - (m+1) cd mod cm has a closed form, so the 64
// lanes make 64 uniforms per round (lanes 33..63 substitute x_{m-33} =
// x_{m-130} - x_{m-66}).  The lanes then take Gaussian1's polar pairs
// (uniforms 2p, 2p+1, RandUtils.f90:156-178) 32 at a time, and the accepted
// pairs are placed by a ballot prefix in stream order (v2 fac, then the saved
// deviate v1 fac).  Nothing is committed until the rotation is done; then the
// state advances by exactly the uniforms the consumed Gaussians used (ring,
// i97/j97, c, iset, gset): bit-identical to drawing them one at a time.
//
// Gram-Schmidt.  Lane j owns row j's vec in registers.  Row i is final once
// its projections on rows 0..i-1 are done, so the rows advance in lockstep:
// at iteration i lane i takes its norm (below 1e-3 row i is redrawn and the
// later rows restart on the shifted Gaussians) and publishes R(i,:) in LDS,
// then every lane j > i projects onto it.  Every sum runs over q in order, as
// the reference's sum() and rot_matrix do, so R is bit-identical.  A rotation
// whose Gaussians would overflow the LDS buffers (many redraws) is redone by
// the serial path (lane 0 draws, the lanes project with readlane sums), which
// is also the debug reference (DevCfg::rot_serial).

// sum of x over lanes 0..n-1 in lane order, formed identically on every lane
// from v_readlane broadcasts (no LDS round trip, no divergent lane-0 section)
__device__ __forceinline__ double lane_sum_ordered(double x, int n)
{
    const long long bits = __double_as_longlong(x);
    const int lo = (int)bits, hi = (int)(bits >> 32);
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < MAXBLK; q++)
        if (q < n) {
            const unsigned l = (unsigned)__builtin_amdgcn_readlane(lo, q);
            const long long h = __builtin_amdgcn_readlane(hi, q);
            s += __longlong_as_double((h << 32) | l);
        }
    return s;
}

__device__ __forceinline__ double readlane_f64(double x, int q)
{
    const long long bits = __double_as_longlong(x);
    const unsigned l = (unsigned)__builtin_amdgcn_readlane((int)bits, q);
    const long long h = __builtin_amdgcn_readlane((int)(bits >> 32), q);
    return __longlong_as_double((h << 32) | l);
}

// LDS written by some lanes of a wave and read by others (the wave's LDS
// operations complete in order; this keeps the compiler from moving them)
__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

static constexpr int ROT_WAVES = 4;                        // walkers per rot_kernel workgroup (a wave each)
static constexpr int ROT_GC = MAXBLK * (MAXBLK + 4);       // Gaussians a parallel rotation may use (>= n (n + ROT_SPEC))
static constexpr int ROT_GA = ROT_GC + 128;                // + one pair round's overshoot
static constexpr int ROT_UC = 1536;                        // uniforms (a multiple of 64)

struct RotLds {
    double g[ROT_GA];             // the Gaussian stream from the rotation's start (g[0] = gset if iset)
    double rm[MAXBLK * MAXBLK];   // R(i, q) at rm[i * MAXBLK + q]
    double u[98];                 // RANMAR u(1:97) as doubles (the state rows' form)
    double gs[MAXBLK];            // serial path: one attempt's Gaussians
    int x[ROT_UC];                // lagged-Fibonacci values x_m (units of 2^-24)
    int o[ROT_UC];                // uniforms x_m - c_m (units of 2^-24)
    int pi[ROT_GA / 2];           // pair index of the r-th accepted pair
    int ui[100];                  // u(1:97) in units of 2^-24
};

struct RotGen {
    int i97, j97, C0;             // RANMAR pointers and carry (units of 2^-24) at the start
    int off;                      // 1 when the start state holds a saved deviate (iset)
    int m = 0, p = 0, nr = 0;     // uniforms made, pairs taken, pairs accepted
    int cbase;                    // carry before this round's first call: C0 - m cd mod cm
    int ck;                       // this lane's (lane + 1) cd mod cm
};

__device__ __forceinline__ int mod97(int v) { return v >= 97 ? v - 97 : v; }   // v in [0, 194)

__device__ __forceinline__ int rot_x(const RotLds &L, const RotGen &G, int p)
{   // x_p; p in [-97, -1] is the start ring: u(i97 - 1 - p mod 97)
    return p >= 0 ? L.x[p] : L.ui[mod97(G.i97 - 1 - p)];
}

__device__ __forceinline__ int sub24(int a, int b) { const int d = a - b; return d < 0 ? d + (1 << 24) : d; }

static constexpr int RM_P = 16777213, RM_CD = 7654321;     // cm and cd in units of 2^-24

__device__ void rot_uniforms(RotLds &L, RotGen &G, int lane)
{   // 64 uniforms
    const int m = G.m + lane;
    const int b = lane < 33 ? rot_x(L, G, m - 33) : sub24(rot_x(L, G, m - 130), rot_x(L, G, m - 66));
    const int x = sub24(rot_x(L, G, m - 97), b);
    int cm = G.cbase - G.ck;                 // c after call m: C0 - (m + 1) cd mod cm
    if (cm < 0) cm += RM_P;
    L.x[m] = x;
    L.o[m] = sub24(x, cm);
    G.m += 64;
    G.cbase -= (64 * RM_CD) % RM_P;
    if (G.cbase < 0) G.cbase += RM_P;
    wave_sync();
}

__device__ void rot_pairs(RotLds &L, RotGen &G, int lane)
{   // up to 64 polar pairs of the uniforms made so far
    const int p = G.p + lane;
    bool acc = false;
    double v1 = 0.0, v2 = 0.0, rr = 0.0;
    if (2 * p < G.m) {
        v1 = 2.0 * ((double)L.o[2 * p] * (1.0 / 16777216.0)) - 1.0;
        v2 = 2.0 * ((double)L.o[2 * p + 1] * (1.0 / 16777216.0)) - 1.0;
        rr = v1 * v1 + v2 * v2;
        acc = rr < 1.0;
    }
    const unsigned long long mask = __ballot(acc);
    if (acc) {
        const int r = G.nr + __popcll(mask & ((1ull << lane) - 1ull));
        const double fac = sqrt(-2.0 * log(rr) / rr);
        L.g[G.off + 2 * r] = v2 * fac;
        L.g[G.off + 2 * r + 1] = v1 * fac;
        L.pi[r] = p;
    }
    G.nr += __popcll(mask);
    G.p = min(G.p + 64, G.m / 2);
    wave_sync();
}

// Gaussians g[0, need): the uniforms for about 1.3 pairs per missing
// accepted pair go first (their rounds are short), then the pairs 64 at a time
__device__ __forceinline__ bool rot_fill(RotLds &L, RotGen &G, int need, int lane)
{
    if (need > ROT_GC) return false;
    while (G.off + 2 * G.nr < need) {
        const int short_pairs = (need - G.off - 2 * G.nr + 1) / 2;
        int want = 2 * (G.p + short_pairs + short_pairs / 3 + 8);
        want = min(ROT_UC, (want + 63) & ~63);
        if (want <= G.m) {
            if (2 * G.p < G.m) want = G.m;        // pairs left to take
            else if (G.m + 64 <= ROT_UC) want = G.m + 64;
            else return false;                    // the uniform buffer is spent
        }
        while (G.m < want) rot_uniforms(L, G, lane);
        while (2 * G.p < G.m && G.off + 2 * G.nr < need) rot_pairs(L, G, lane);
    }
    return true;
}

// advance the RANMAR / Gaussian1 state past the first T Gaussians of the stream
__device__ void rot_commit(RotLds &L, const RotGen &G, int T, Rng &r, int lane)
{
    const int t = T - G.off;
    int K = 0;
    if (t > 0) {
        const int q = (t - 1) / 2;            // the pair that gave the last Gaussian
        K = 2 * (L.pi[q] + 1);
        r.iset = t & 1;
        r.gset = L.g[G.off + 2 * q + 1];
    } else {
        r.iset = 0;
    }
    for (int s = lane; s < 97; s += 64) {    // ring slot s (u(s+1)) last written by call m = i97-1-s mod 97 (+97k)
        const int r0 = mod97(G.i97 - 1 - s + 97);
        if (K - 1 >= r0) L.ui[s] = L.x[r0 + 97 * ((K - 1 - r0) / 97)];
        L.u[s] = (double)L.ui[s] * (1.0 / 16777216.0);
    }
    r.i97 = (G.i97 - 1 - K % 97 + 97) % 97 + 1;
    r.j97 = (G.j97 - 1 - K % 97 + 97) % 97 + 1;
    int cm = G.C0 - (int)((long long)K * RM_CD % RM_P);
    if (cm < 0) cm += RM_P;
    r.c = (double)cm * (1.0 / 16777216.0);
    wave_sync();
}

#ifdef CMAMD_STAMPS
__device__ unsigned long long g_rot_ticks[3];     // first listed walker: total, Gaussian draws, Gram-Schmidt
#define RTICK(v) (v) = __builtin_amdgcn_s_memtime()
#else
#define RTICK(v) ((void)0)
#endif

static constexpr int ROT_SPEC = 2;   // idle lanes n, n+1 carry the last row's next two attempts

// One lockstep Gram-Schmidt pass over rows start..n-1 (row j from the n
// Gaussians at g[gbase + (j - start) n]); NQ = n rounded up to 8.  The
// padding columns q in [n, NQ) hold +0.0 in vec and in R, so every product
// there is +0.0 and the sums (which start at +0.0) are bit-identical to sums
// over q < n, with no selects.  Lane i publishes its raw vec and the lanes
// divide one element each.  A redraw is most likely for the last row (its
// residual has one degree of freedom: P(norm <= 1e-3) = 2.5 %), so lanes n and
// n+1 project the Gaussians that follow as that row's second and third
// attempts and stand in when it fails.  Returns -1 and the last row's extra
// attempts in *extra, or the row to redraw and its failed attempts in *extra.
template <int NQ>
__device__ int rot_gs_pass(RotLds &L, int n, int start, int gbase, int lane, int spec, int *extra)
{
    const int top = n + spec;
    double v[NQ], pp[NQ];
    if (lane >= start && lane < top) {
        const double *gv = L.g + gbase + (lane - start) * n;   // within g: the fill covered (top - start) n
#pragma unroll
        for (int q = 0; q < NQ; q++) {
            const double x = gv[q];
            v[q] = q < n ? x : 0.0;
        }
    }
    for (int i = 0; i < n; i++) {
        if (i >= start) {
            const bool last = i == n - 1;
            double norm = 0.0;
            if (lane == i || (last && lane >= n && lane < top)) {
#pragma unroll
                for (int q = 0; q < NQ; q++) pp[q] = v[q] * v[q];
#pragma unroll
                for (int q = 0; q < NQ; q++) norm += pp[q];
            }
            int src = i, a = 0;
            double nv = readlane_f64(norm, i);
            if (!(nv > 1e-3)) {               // RandRotationD :143: draw row i again
                if (!last) {
                    *extra = 1;
                    return i;
                }
                for (a = 1; a <= spec; a++) {
                    nv = readlane_f64(norm, n - 1 + a);
                    if (nv > 1e-3) break;
                }
                if (a > spec) {
                    *extra = 1 + spec;
                    return i;
                }
                src = n - 1 + a;
            }
            *extra = a;
            double *ri = L.rm + i * MAXBLK;
            if (lane == src)
#pragma unroll
                for (int q = 0; q < NQ; q += 2) *reinterpret_cast<double2 *>(ri + q) = make_double2(v[q], v[q + 1]);
            wave_sync();
            if (lane < NQ) {                  // R(i, q) = vec(q) / sqrt(norm), lane q
                const double x = ri[lane];
                ri[lane] = lane < n ? x / sqrt(nv) : 0.0;
            }
            wave_sync();
        }
        if (i < n - 1 && lane > i && lane < top) {   // vec = vec - sum(vec*R(i,:))*R(i,:)
            const double *ri = L.rm + i * MAXBLK;
            double rv[NQ];
#pragma unroll
            for (int q = 0; q < NQ; q += 2) {
                const double2 t = *reinterpret_cast<const double2 *>(ri + q);
                rv[q] = t.x;
                rv[q + 1] = t.y;
            }
#pragma unroll
            for (int q = 0; q < NQ; q++) pp[q] = v[q] * rv[q];
            double s = 0.0;
#pragma unroll
            for (int q = 0; q < NQ; q++) s += pp[q];
#pragma unroll
            for (int q = 0; q < NQ; q++) pp[q] = s * rv[q];
#pragma unroll
            for (int q = 0; q < NQ; q++) v[q] = v[q] - pp[q];
        }
    }
    return -1;
}

// the parallel rotation into L.rm; false (state untouched) when the buffers overflow
__device__ bool rot_parallel(RotLds &L, Rng &r, int n, int lane, int spec, unsigned long long *tk)
{
    RotGen G;
    G.i97 = r.i97;
    G.j97 = r.j97;
    G.C0 = (int)(r.c * 16777216.0);
    G.off = r.iset ? 1 : 0;
    G.cbase = G.C0;
    G.ck = (lane + 1) * RM_CD % RM_P;                      // < 64 cd < 2^31
    if ((G.i97 - G.j97 + 97) % 97 != 64) return false;     // not RMARIN's pointer pair: serial path
    for (int s = lane; s < 97; s += 64) L.ui[s] = (int)(L.u[s] * 16777216.0);
    if (lane == 0 && G.off) L.g[0] = r.gset;
    wave_sync();
    int start = 0, gbase = 0;
    (void)tk;
    for (;;) {                                // one pass per redraw
#ifdef CMAMD_STAMPS
        unsigned long long t0, t1;
        RTICK(t0);
#endif
        if (!rot_fill(L, G, gbase + (n - start + spec) * n, lane)) return false;
#ifdef CMAMD_STAMPS
        RTICK(t1);
        tk[1] += t1 - t0;
#endif
        int extra = 0;
        const int fail = n <= 8    ? rot_gs_pass<8>(L, n, start, gbase, lane, spec, &extra)
                         : n <= 16 ? rot_gs_pass<16>(L, n, start, gbase, lane, spec, &extra)
                         : n <= 24 ? rot_gs_pass<24>(L, n, start, gbase, lane, spec, &extra)
                                   : rot_gs_pass<32>(L, n, start, gbase, lane, spec, &extra);
        static_assert(MAXBLK == 32, "rot_gs_pass widths");
#ifdef CMAMD_STAMPS
        RTICK(t0);
        tk[2] += t0 - t1;
#endif
        if (fail < 0) {
            rot_commit(L, G, gbase + (n - start + extra) * n, r, lane);
            return true;
        }
        gbase += (fail - start + extra) * n;
        start = fail;
    }
}

// the serial rotation into L.rm: lane 0 draws each attempt's Gaussians, lane q
// holds column q of R, every sum is formed in q order from readlane broadcasts
__device__ void rot_serial(RotLds &L, Rng &r, int n, int lane)
{
    double rcol[MAXBLK];
#pragma unroll
    for (int i = 0; i < MAXBLK; i++) rcol[i] = 0.0;
    for (int j = 0; j < n; j++) {
        double v, norm;
        for (;;) {
            if (lane == 0)
                for (int q = 0; q < n; q++) L.gs[q] = gaussian1(r);
            wave_sync();
            v = lane < n ? L.gs[lane] : 0.0;
#pragma unroll
            for (int i = 0; i < MAXBLK; i++) {
                if (i < j) {
                    const double s = lane_sum_ordered(v * rcol[i], n);
                    v = v - s * rcol[i];
                }
            }
            norm = lane_sum_ordered(v * v, n);
            wave_sync();
            if (norm > 1e-3) break;
        }
        const double rv = v / sqrt(norm);
#pragma unroll
        for (int i = 0; i < MAXBLK; i++)
            if (i == j) rcol[i] = rv;
        if (lane < n) L.rm[j * MAXBLK + lane] = rv;
    }
    // lane 0's RNG state is the walker's: broadcast it
    r.c = readlane_f64(r.c, 0);
    r.gset = readlane_f64(r.gset, 0);
    r.i97 = __builtin_amdgcn_readlane(r.i97, 0);
    r.j97 = __builtin_amdgcn_readlane(r.j97, 0);
    r.iset = __builtin_amdgcn_readlane(r.iset, 0);
    wave_sync();
}

// One wave: walker w's pending rotation, then the rest of its proposal.
__device__ void rot_walker(const DevCfg &c, int w, int lane, RotLds &L, bool stamp)
{
    const size_t ld = c.ld;
    const Rows &R = c.rows;
    const int b = c.si[(size_t)R.PROT * ld + w] - 1;
    const Tabs t = make_tabs(c, c.tab_i, c.tab_d, c.tab_d);
    const int n = t.blk_n[b], off = t.blk_R_off[b];
    for (int i = lane; i < 97; i += 64) L.u[i] = c.sd[(size_t)(R.U + i) * ld + w];
    Walker k;
    k.r.u = Col<double>{L.u, 1};
    k.r.c = c.sd[(size_t)R.C * ld + w];
    k.r.gset = c.sd[(size_t)R.G * ld + w];
    k.r.i97 = c.si[(size_t)R.I97 * ld + w];
    k.r.j97 = c.si[(size_t)R.J97 * ld + w];
    k.r.iset = c.si[(size_t)R.ISET * ld + w];
    wave_sync();
    unsigned long long tk[3] = {0, 0, 0};
#ifdef CMAMD_STAMPS
    RTICK(tk[0]);
#endif
    if (c.rot_serial == 1 || !rot_parallel(L, k.r, n, lane, c.rot_serial == 2 ? 0 : ROT_SPEC, tk))
        rot_serial(L, k.r, n, lane);
#ifdef CMAMD_STAMPS
    if (stamp && lane == 0) {
        g_rot_ticks[0] = __builtin_amdgcn_s_memtime() - tk[0];
        g_rot_ticks[1] = tk[1];
        g_rot_ticks[2] = tk[2];
    }
#else
    (void)stamp;
#endif
    // R(i, q) (rm, row stride MAXBLK) -> the state rows and a packed copy (row stride n) in g
    for (int e = lane; e < n * n; e += 64) {
        const double x = L.rm[(e / n) * MAXBLK + e % n];
        c.sd[(size_t)(R.R + off + e) * ld + w] = x;
        L.g[e] = x;
    }
    wave_sync();
    k.trial = Col<double>{c.sd + (size_t)R.T * ld + w, (int)ld};
    k.P = Col<double>{c.sd + (size_t)R.P * ld + w, (int)ld};
    if (lane == 0) {   // the rest of ProposeVec on column 1 of the packed copy of R, up to UpdateParams
        k.R = Col<double>{L.g - off, 1};
        k.vec = Col<double>{L.gs, 1};
        k.blklp = Col<int>{c.si + (size_t)R.BLKLP * ld + w, (int)ld};
        k.defer = 1;
        proposal_tail(c, t, k, b, 0);
    }
    wave_sync();
    {   // UpdateParams (propose.f90:142-149): one lane per changed parameter, each sum in q order
        const int nc = t.blk_nchanged[b];
        const double *M = t.mapping + t.blk_map_off[b];
        const int *chg = t.changed + t.blk_changed_off[b];
        for (int j = lane; j < nc; j += 64) {
            double s = 0.0;
            for (int q = 0; q < n; q++) s += M[j * n + q] * L.gs[q];
            k.trial[chg[j]] += s;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");   // the trial row's stores, before lane 0 reads it
    __builtin_amdgcn_wave_barrier();
    double calr = 0.0;   // bin co-run: plik's trial calibration
    if (lane == 0) {
        for (int l = 0; l < c.n_like; l++)
            for (int q = 0; q < c.like_nn[l]; q++)
                c.like_nuis[l][(size_t)w * c.like_nn[l] + q] = k.trial[t.ti[c.like_nidx[l] + q]];
        if (c.bin_on) calr = k.trial[t.ti[c.like_nidx[0] + c.bin_cal]];
        if (c.mask_on) write_like_flags(c, k.trial, k.P, w);
        c.sd[(size_t)R.C * ld + w] = k.r.c;
        c.sd[(size_t)R.G * ld + w] = k.r.gset;
        c.si[(size_t)R.I97 * ld + w] = k.r.i97;
        c.si[(size_t)R.J97 * ld + w] = k.r.j97;
        c.si[(size_t)R.ISET * ld + w] = k.r.iset;
        c.si[(size_t)R.PROT * ld + w] = 0;
    }
    wave_sync();
    for (int i = lane; i < 97; i += 64) c.sd[(size_t)(R.U + i) * ld + w] = L.u[i];
    if (c.bin_on) {   // the walker's Delta rows from the bin co-run's raw sums (plik_bin_emit's operations)
        const double cl = __shfl(calr, 0), c2 = cl * cl;
        const size_t r = (size_t)w * c.bin_Np;
#pragma unroll 4
        for (int i = lane; i < c.bin_nused; i += 64) c.bin_delta[r + i] = c.bin_X[i] - c.bin_S[r + i] / c2;
    }
}

// One wave per listed walker (the launch's list counter is wave-uniform).
__global__ __launch_bounds__(64 * ROT_WAVES) void rot_kernel(DevCfg c, int g0)
{
    extern __shared__ __attribute__((aligned(16))) double rot_lds[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int idx = blockIdx.x * ROT_WAVES + wave;
    if (idx >= c.rot_cnt[2 * (g0 / 64) + c.rot_par]) return;
    rot_walker(c, c.rot_list[g0 + idx], lane, reinterpret_cast<RotLds *>(rot_lds)[wave], idx == 0);
}

#ifdef CMAMD_STAMPS
extern "C" int cmamd_debug_rot_ticks(unsigned long long *host) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_rot_ticks), sizeof(g_rot_ticks)) == hipSuccess ? 0 : -5;
}
#endif

// ---------------------------------------------------------------- fast dragging
// TFastDraggingSampler_GetNewSample (MCMC.f90:338-452) in four launch stages,
// one thread per walker on the walker state in HBM (the drag scratch lives in
// separate rows, DragCfg::dd / di, so the Metropolis kernel's LDS image is
// unchanged).  Between stages the host evaluates the likelihoods:
//   set 1 at the trial-end rows T on the END slow point's theory,
//   set 2 at the trial-start rows T2 on the walker's current theory.
//   stage 0  TrialEnd = Cur + GetProposalSlow                        (:367-368)
//   stage 1  CurEndLike; abort on logZero (:370-374); first delta    (:386-394)
//   stage 2  interpolated Metropolis on (start, end) likes, sums; next delta,
//            or (last step) the drag accept + MoveDone                (:395-452)
// dst: 0 idle, 1 dragging, 2 aborted, 3 skipped (CurLike == logZero),
//      4 accepted (the walker's theory must become the end theory)
struct DragCfg {
    double *dd;      // [3 np + 4 + max_blk + n_like][ld]: CE, CS, T2, (cel, csl, ss, se), vec scratch,
                     //   per-likelihood terms at CE
    int *di;         // [1 + all_n][ld]: dst, RandIndices scratch
    int interp, istep;
    const double *like_terms2;            // [n_like][ld] at T2
    double *like_nuis2[MAXLIKE];          // [W][nn] DataParams at T2
};

// One walker's part of a drag stage (TFastDraggingSampler_GetNewSample,
// MCMC.f90:338-452) on views of its state: in HBM (drag_kernel) or in an LDS
// image (drag_staged_kernel).  STAGE 0 proposes the slow trial, 1 scores the
// end point, 2 runs interpolation step g.istep.
struct DragView {
    Col<double> T, CE, CS, T2, ET, lk1, lk2;
    double *cur, *mult, *cel, *csl, *ss, *se;
    int *nacc, *dst;
};

template <int STAGE>
__device__ __forceinline__ void drag_logic(const DevCfg &c, const DragCfg &g, const Tabs &t, Walker &k,
                                           const DragView &v, int w, double *hist_row, double *hist_terms)
{
    const size_t ld = c.ld;
    const int np = c.np;
    const Col<double> T = v.T, CE = v.CE, CS = v.CS, T2 = v.T2, ET = v.ET, lk1 = v.lk1, lk2 = v.lk2;
    double &cur = *v.cur;
    double &mult = *v.mult;
    int &nacc = *v.nacc;
    double &cel = *v.cel;
    double &csl = *v.csl;
    double &ss = *v.ss;
    double &se = *v.se;
    int &dst = *v.dst;
    auto keep_end_terms = [&]() {
        for (int l = 0; l < c.n_like; l++) ET[l] = lk1[l];
    };

    auto scatter = [&]() {            // DataParams of both trial points
        for (int l = 0; l < c.n_like; l++)
            for (int q = 0; q < c.like_nn[l]; q++) {
                c.like_nuis[l][(size_t)w * c.like_nn[l] + q] = T[t.ti[c.like_nidx[l] + q]];
                g.like_nuis2[l][(size_t)w * c.like_nn[l] + q] = T2[t.ti[c.like_nidx[l] + q]];
            }
    };
    auto next_delta = [&]() {         // GetProposalFastDelta (propose.f90:291-298) on both ends
        Col<double> keep = k.trial;
        for (int i = 0; i < np; i++) T2[i] = 0.0;
        k.trial = T2;
        proposal_fast(c, t, k);
        k.trial = keep;
        for (int i = 0; i < np; i++) {
            const double d = T2[i];
            T[i] = CE[i] + d;
            T2[i] = CS[i] + d;
        }
    };
    auto metropolis = [&](double like, double curl) {   // MCMC.f90:119-131
        if (like == LOGZERO) return false;
        bool a = curl > like;
        if (!a) a = (double)randexp1(k.r) > like - curl;
        return a;
    };

    if (STAGE == 0) {
        if (cur == LOGZERO) {
            dst = 3;
        } else {
            dst = 1;
            for (int i = 0; i < np; i++) {
                T[i] = k.P[i];
                CS[i] = k.P[i];
                T2[i] = k.P[i];
            }
            csl = cur;
            proposal_slow(c, t, k);
        }
        scatter();
    } else if (STAGE == 1) {
        if (dst == 1) {
            cel = target_like(c, t, T, lk1);
            if (cel == LOGZERO) {
                dst = 2;
                mult += 1.0;
            } else {
                for (int i = 0; i < np; i++) CE[i] = T[i];
                keep_end_terms();
                ss = csl;
                se = cel;
                next_delta();
            }
        }
        scatter();
    } else {
        if (dst == 1) {
            const double el = target_like(c, t, T, lk1);
            bool acc = el != LOGZERO;
            double sl = 0.0;
            if (acc) {
                sl = target_like(c, t, T2, lk2);
                acc = sl != LOGZERO;
                if (acc) {
                    const double frac = (double)g.istep / g.interp;
                    const double cint = csl * (1 - frac) + frac * cel;
                    const double ilike = sl * (1 - frac) + frac * el;
                    acc = metropolis(ilike, cint);
                }
            }
            if (acc) {
                for (int i = 0; i < np; i++) {
                    CE[i] = T[i];
                    CS[i] = T2[i];
                }
                cel = el;
                csl = sl;
                keep_end_terms();
            }
            ss = ss + csl;
            se = se + cel;
            if (g.istep < g.interp - 1) {
                next_delta();
            } else {
                const double cur_drag = ss / g.interp, drag = se / g.interp;
                if (metropolis(drag, cur_drag)) {        // MoveDone :166-190 + :437-445
                    if (mult > 0) nacc += 1;
                    mult = 1.0;
                    for (int i = 0; i < np; i++) k.P[i] = CE[i];
                    cur = cel;
                    for (int l = 0; l < c.n_like; l++) c.cur_terms[(size_t)l * ld + w] = ET[l];
                    dst = 4;
                } else {
                    mult += 1.0;
                    dst = 0;
                }
            }
        }
        if (g.istep < g.interp - 1) {
            scatter();
        } else {
            if (dst == 2 || dst == 3) dst = 0;
            if (hist_row)
            {
                for (int i = 0; i < c.n_used; i++) hist_row[(size_t)i * c.W + w] = k.P[t.params_used[i]];
                hist_row[(size_t)c.n_used * c.W + w] = cur;
            }
            if (hist_terms)
                for (int l = 0; l < c.n_like; l++) hist_terms[(size_t)l * c.W + w] = c.cur_terms[(size_t)l * ld + w];
        }
    }
}

template <int STAGE>
__global__ __launch_bounds__(64) void drag_kernel(DevCfg c, DragCfg g, double *hist_row, double *hist_terms)
{
    const int w = blockIdx.x * 64 + threadIdx.x;
    if (w >= c.W) return;
    const size_t ld = c.ld;
    const Rows &R = c.rows;
    const int np = c.np;
    auto drow = [&](double *b, int r) { return Col<double>{b + (size_t)r * ld + w, (int)ld}; };
    auto irow = [&](int *b, int r) { return Col<int>{b + (size_t)r * ld + w, (int)ld}; };
    const Tabs t = make_tabs(c, c.tab_i, c.tab_d);
    Walker k;
    k.r.u = drow(c.sd, R.U);
    k.r.c = c.sd[(size_t)R.C * ld + w];
    k.r.gset = c.sd[(size_t)R.G * ld + w];
    k.r.i97 = c.si[(size_t)R.I97 * ld + w];
    k.r.j97 = c.si[(size_t)R.J97 * ld + w];
    k.r.iset = c.si[(size_t)R.ISET * ld + w];
    k.R = drow(c.sd, R.R);
    k.P = drow(c.sd, R.P);
    k.trial = drow(c.sd, R.T);
    k.vec = drow(g.dd, 3 * np + 4);
    k.cyc = irow(c.si, R.CYC);
    k.cyclp = irow(c.si, R.CYCLP);
    k.blklp = irow(c.si, R.BLKLP);
    k.itmp = irow(g.di, 1);
    k.fast_ix = c.si[(size_t)R.FASTIX * ld + w];
    DragView v;
    v.T = k.trial;
    v.CE = drow(g.dd, 0);
    v.CS = drow(g.dd, np);
    v.T2 = drow(g.dd, 2 * np);
    v.ET = drow(g.dd, 3 * np + 4 + c.max_blk);   // terms at CE
    v.lk1 = Col<double>{const_cast<double *>(c.like_terms) + w, (int)ld};
    v.lk2 = Col<double>{const_cast<double *>(g.like_terms2) + w, (int)ld};
    v.cur = c.sd + (size_t)R.L * ld + w;
    v.mult = c.sd + (size_t)R.M * ld + w;
    v.nacc = c.si + (size_t)R.NACC * ld + w;
    v.cel = g.dd + (size_t)(3 * np + 0) * ld + w;
    v.csl = g.dd + (size_t)(3 * np + 1) * ld + w;
    v.ss = g.dd + (size_t)(3 * np + 2) * ld + w;
    v.se = g.dd + (size_t)(3 * np + 3) * ld + w;
    v.dst = g.di + w;
    drag_logic<STAGE>(c, g, t, k, v, w, hist_row, hist_terms);
    c.sd[(size_t)R.C * ld + w] = k.r.c;
    c.sd[(size_t)R.G * ld + w] = k.r.gset;
    c.si[(size_t)R.I97 * ld + w] = k.r.i97;
    c.si[(size_t)R.J97 * ld + w] = k.r.j97;
    c.si[(size_t)R.ISET * ld + w] = k.r.iset;
    c.si[(size_t)R.FASTIX * ld + w] = k.fast_ix;
}

// The same stage on an LDS image of MB walkers' state (mh_kernel's staging:
// the sampler rows, the drag rows, both likelihood-term sets and the tables by
// LDS-DMA, one wait), so the chain's dependent reads are LDS round trips
// instead of HBM ones; then the image is written back.  Used when the image
// fits (drag_lds_bytes).
__host__ __device__ inline int drag_rows(const DevCfg &c) { return 3 * c.np + 4 + c.max_blk + c.n_like; }

template <int STAGE>
__global__ __launch_bounds__(MH_THREADS) void drag_staged_kernel(DevCfg c, DragCfg g, double *hist_row,
                                                                 double *hist_terms)
{
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const Rows &R = c.rows;
    const int lane = threadIdx.x % MB;
    const int wl64 = threadIdx.x & 63, wave = threadIdx.x >> 6, nwave = MH_THREADS / 64;
    const int wb = blockIdx.x * MB;
    const int w = wb + lane;
    const size_t W = c.ld;
    const int np = c.np;
    const int nlk = (c.n_like + 1) & ~1;            // LDS rows (even); nl, nr of them are moved
    const int nl = c.n_like;
    const int nr = drag_rows(c);
    const int ndd = (nr + 1) & ~1;
    const int nd_st = c.stage_R ? R.ND : R.ND - R.RR;
    const int ni_st = c.stage_cyc ? R.NI : R.CYC;
    const int ntd = c.stage_cov ? c.tl.n_dbl : c.tl.covinv;
    const bool skipR = !c.stage_R;
    double *sd = lds;                                        // [nd_st][MB]
    double *dd = sd + (size_t)nd_st * MB;                    // [ndd][MB] drag rows
    double *l1 = dd + (size_t)ndd * MB;                      // [nlk][MB] terms at T
    double *l2 = l1 + (size_t)nlk * MB;                      // [nlk][MB] terms at T2
    double *td = l2 + (size_t)nlk * MB;                      // [ntd rounded to 32]
    int *si = reinterpret_cast<int *>(td + ((ntd + 31) & ~31));   // [ni_st][MB]
    int *dst_l = si + (size_t)ni_st * MB;                    // [4][MB] dst (row 0)
    int *it = dst_l + 4 * MB;                                // [all_n][MB] RandIndices scratch
    int *ti = it + (size_t)c.all_n * MB;                     // [n_int rounded to 64]
#define SROW(r) ((skipR && (r) >= R.R) ? (r) - R.RR : (r))
    const int rEnd = R.R + R.RR;
    if (skipR) {
        dma_rows_f64(sd, 0, c.sd, 0, R.R, W, wb, wl64, wave, nwave);
        dma_rows_f64(sd, R.R, c.sd, rEnd, R.ND - rEnd, W, wb, wl64, wave, nwave);
    } else {
        dma_rows_f64(sd, 0, c.sd, 0, R.ND, W, wb, wl64, wave, nwave);
    }
    dma_rows_f64(dd, 0, g.dd, 0, nr, W, wb, wl64, wave, nwave);
    dma_rows_f64(l1, 0, c.like_terms, 0, nl, W, wb, wl64, wave, nwave);
    dma_rows_f64(l2, 0, g.like_terms2, 0, nl, W, wb, wl64, wave, nwave);
    dma_rows_i32(si, c.si, ni_st, W, wb, wl64, wave, nwave);
    dma_rows_i32(dst_l, g.di, 1, W, wb, wl64, wave, nwave);
    dma_words(td, c.tab_d, 2 * ntd, wl64, wave, nwave);
    dma_words(ti, c.tab_i, c.tl.n_int, wl64, wave, nwave);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x < MB && w < c.W) {
        const Tabs t = make_tabs(c, ti, td, c.stage_cov ? td : c.tab_d);
        auto lrow = [&](double *b, int r) { return Col<double>{b + (size_t)r * MB + lane, MB}; };
        Walker k;
        k.r.u = lrow(sd, R.U);
        k.r.c = sd[(size_t)R.C * MB + lane];
        k.r.gset = sd[(size_t)R.G * MB + lane];
        k.r.i97 = si[(size_t)R.I97 * MB + lane];
        k.r.j97 = si[(size_t)R.J97 * MB + lane];
        k.r.iset = si[(size_t)R.ISET * MB + lane];
        k.R = c.stage_R ? lrow(sd, R.R) : Col<double>{c.sd + (size_t)R.R * W + w, c.ld};
        k.P = lrow(sd, SROW(R.P));
        k.trial = lrow(sd, SROW(R.T));
        k.vec = lrow(dd, 3 * np + 4);
        k.cyc = c.stage_cyc ? Col<int>{si + (size_t)R.CYC * MB + lane, MB} : Col<int>{c.si + (size_t)R.CYC * W + w, c.ld};
        k.cyclp = Col<int>{si + (size_t)R.CYCLP * MB + lane, MB};
        k.blklp = Col<int>{si + (size_t)R.BLKLP * MB + lane, MB};
        k.itmp = Col<int>{it + lane, MB};
        k.fast_ix = si[(size_t)R.FASTIX * MB + lane];
        DragView v;
        v.T = k.trial;
        v.CE = lrow(dd, 0);
        v.CS = lrow(dd, np);
        v.T2 = lrow(dd, 2 * np);
        v.ET = lrow(dd, 3 * np + 4 + c.max_blk);
        v.lk1 = lrow(l1, 0);
        v.lk2 = lrow(l2, 0);
        v.cur = sd + (size_t)SROW(R.L) * MB + lane;
        v.mult = sd + (size_t)SROW(R.M) * MB + lane;
        v.nacc = si + (size_t)R.NACC * MB + lane;
        v.cel = dd + (size_t)(3 * np + 0) * MB + lane;
        v.csl = dd + (size_t)(3 * np + 1) * MB + lane;
        v.ss = dd + (size_t)(3 * np + 2) * MB + lane;
        v.se = dd + (size_t)(3 * np + 3) * MB + lane;
        v.dst = dst_l + lane;
        const int i97_0 = k.r.i97;
        drag_logic<STAGE>(c, g, t, k, v, w, hist_row, hist_terms);
        dst_l[MB + lane] = k.r.nd < 97 ? k.r.nd : 97;   // rows 1, 2: the ring entries the draws overwrote
        dst_l[2 * MB + lane] = i97_0;
        sd[(size_t)R.C * MB + lane] = k.r.c;
        sd[(size_t)R.G * MB + lane] = k.r.gset;
        si[(size_t)R.I97 * MB + lane] = k.r.i97;
        si[(size_t)R.J97 * MB + lane] = k.r.j97;
        si[(size_t)R.ISET * MB + lane] = k.r.iset;
        si[(size_t)R.FASTIX * MB + lane] = k.fast_ix;
    }
    __syncthreads();
    // of the RANMAR ring only the entries this stage's draws overwrote
    // (positions i97 - 1, i97 - 2, ... mod 97 of the first index), as mh_body:
    // the stages 63.4-63.8 against 63.8-67.4 us a drag step (round 6, tools/gpu_r6u.sh)
    if (w < c.W) {
        const int nd = dst_l[MB + lane], i0 = dst_l[2 * MB + lane];
        for (int q = threadIdx.x / MB; q < nd; q += NV) {
            int p = i0 - 1 - q;
            if (p < 0) p += 97;
            c.sd[(size_t)(R.U + p) * W + w] = sd[(size_t)(R.U + p) * MB + lane];
        }
    }
    if (skipR) {
        stage_out(c.sd, sd, R.C, R.C, R.R, W, wb);
        stage_out(c.sd, sd, R.R, rEnd, R.ND, W, wb);
    } else {
        stage_out(c.sd, sd, R.C, R.C, R.ND, W, wb);
    }
    stage_out(g.dd, dd, 0, 0, nr, W, wb);
    stage_out(c.si, si, 0, 0, ni_st, W, wb);
    stage_out(g.di, dst_l, 0, 0, 1, W, wb);
#undef SROW
}

// accepted moves: the trial (end) slow point's theory becomes the walker's theory
// (flag[w] == value: drag_kernel dst 4, or the Metropolis accept flag row)
__global__ void drag_swap_theory(const int *flag, int value, int W, const double *src, long long src_ld,
                                 double *dstth, long long dst_ld, long long n)
{
    const int w = blockIdx.y;
    if (w >= W || flag[w] != value) return;
    const double *a = src + (long long)w * src_ld;
    double *d = dstth + (long long)w * dst_ld;
    const long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x, stride = (long long)gridDim.x * blockDim.x;
    if (((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(d)) & 15) == 0) {   // 16-byte moves
        const long long n2 = n / 2;
        for (long long i = t; i < n2; i += stride)
            reinterpret_cast<double2 *>(d)[i] = reinterpret_cast<const double2 *>(a)[i];
        if (t == 0 && (n & 1)) d[n - 1] = a[n - 1];
    } else {
        for (long long i = t; i < n; i += stride) d[i] = a[i];
    }
}

// Starting point: -lnL of P = trial (likelihood terms already evaluated)
__global__ void start_kernel(DevCfg c)
{
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= c.W) return;
    const size_t W = c.ld;
    const Tabs t = make_tabs(c, c.tab_i, c.tab_d);
    Col<double> q{c.sd + (size_t)c.rows.T * W + w, c.ld};
    Col<const double> lk{c.like_terms + w, c.ld};
    c.sd[(size_t)c.rows.L * W + w] = target_like(c, t, q, lk);
    for (int l = 0; l < c.n_like; l++) c.cur_terms[(size_t)l * W + w] = lk[l];
    for (int i = 0; i < c.np; i++) c.sd[(size_t)(c.rows.P + i) * W + w] = q[i];
    c.sd[(size_t)c.rows.M * W + w] = 0.0;
    c.si[(size_t)c.rows.NACC * W + w] = 0;
}

// DataParams of every walker's trial point, P(nuisance_indices)
// (GeneralTypes.f90:642-646, calclike.f90:380): out[w][k] = trial[nidx[k]][w]
__global__ void gather_nuis(const double *trial, int W, int ld, const int *nidx, int n_nuis, double *out)
{
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= W) return;
    for (int k = 0; k < n_nuis; k++) out[(size_t)w * n_nuis + k] = trial[(size_t)nidx[k] * ld + w];
}

// Change mask, sparse likelihoods: the walkers whose flag is set get compact
// slots in walker order (a deterministic block scan; one 1024-thread block per
// sparse likelihood); the flag becomes slot + 1, slot -> walker goes to map,
// the walker's DataParams row is copied to its slot, and cnt[b] is the count.
struct SparseSet {
    int like[MAXLIKE], nn[MAXLIKE];
    double *nuisc[MAXLIKE];
    int *map[MAXLIKE];
};

__global__ __launch_bounds__(1024) void like_compact_kernel(DevCfg c, SparseSet ss, int *__restrict__ cnt)
{
    __shared__ int wsum[16];
    const int b = blockIdx.x, l = ss.like[b], nn = ss.nn[b];
    int *flag = c.like_flag + (size_t)l * c.ld;
    const double *nuis = c.like_nuis[l];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int chunk = (c.W + 1023) / 1024, w0 = t * chunk, w1 = min(c.W, w0 + chunk);
    int n = 0;
    for (int w = w0; w < w1; w++) n += flag[w] != 0;
    int v = n;                                       // inclusive scan: wave, then the 16 wave totals
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(v, o);
        if (lane >= o) v += y;
    }
    if (lane == 63) wsum[wave] = v;
    __syncthreads();
    int before = 0;
    for (int q = 0; q < wave; q++) before += wsum[q];
    int off = before + v - n;
    for (int w = w0; w < w1; w++)
        if (flag[w] != 0) {
            flag[w] = off + 1;
            ss.map[b][off] = w;
            for (int q = 0; q < nn; q++) ss.nuisc[b][(size_t)off * nn + q] = nuis[(size_t)w * nn + q];
            off++;
        }
    if (t == 1023) cnt[b] = before + v;
}

// theory rows of the compacted walkers (sparse likelihood with per-walker theory)
__global__ __launch_bounds__(256) void gather_theory_kernel(const double *__restrict__ dl, long long ld_walker,
                                                            long long ext, const int *__restrict__ map,
                                                            const int *__restrict__ cnt, double *__restrict__ dlc)
{
    const int w = blockIdx.x;
    if (w >= *cnt) return;
    const double *src = dl + (long long)map[w] * ld_walker;
    double *dst = dlc + (long long)w * ld_walker;
    for (long long i = threadIdx.x; i < ext; i += 256) dst[i] = src[i];
}

// Per-chain mean and covariance over history rows first..last
// (SampleCollector.f90:235-246), two passes like the reference (mean, then
// the centred products).  A block owns 64 walkers (lane = walker, coalesced
// rows) and HS_PH row phases (wave p takes rows first+p, first+p+HS_PH, ...);
// the phase partials are combined in fixed order, so results are
// deterministic.  The covariance pass runs one block per (walker tile,
// parameter i) with the n products of row i in registers (NC = n rounded up).
static constexpr int HS_PH = 4;

template <int NC>
__global__ __launch_bounds__(64 * HS_PH) void hist_mean_kernel(const double *hist, int cap, int W, int n, int first,
                                                              int last, double *means)
{
    __shared__ double part[HS_PH][NC][64];
    const int lane = threadIdx.x & 63, ph = threadIdx.x >> 6;
    const int w = blockIdx.x * 64 + lane;
    double acc[NC];
#pragma unroll
    for (int j = 0; j < NC; j++) acc[j] = 0.0;
    if (w < W)
        for (int tt = first + ph; tt <= last; tt += HS_PH) {
            const double *row = hist + (size_t)(tt % cap) * (n + 1) * W + w;
#pragma unroll
            for (int j = 0; j < NC; j++)
                if (j < n) acc[j] += row[(size_t)j * W];
        }
#pragma unroll
    for (int j = 0; j < NC; j++) part[ph][j][lane] = acc[j];
    __syncthreads();
    if (ph == 0 && w < W) {
        const double cnt = last - first + 1;
        for (int j = 0; j < n; j++) {
            double v = part[0][j][lane];
            for (int p = 1; p < HS_PH; p++) v += part[p][j][lane];
            means[(size_t)w * n + j] = v / cnt;
        }
    }
}

template <int NC>
__global__ __launch_bounds__(64 * HS_PH) void hist_cov_kernel(const double *hist, int cap, int W, int n, int first,
                                                             int last, const double *means, double *covs)
{
    __shared__ double part[HS_PH][NC][64];
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
    if (w < W)
        for (int tt = first + ph; tt <= last; tt += HS_PH) {
            const double *row = hist + (size_t)(tt % cap) * (n + 1) * W + w;
            const double di = row[(size_t)i * W] - mi;
#pragma unroll
            for (int j = 0; j < NC; j++)
                if (j < n) acc[j] += (row[(size_t)j * W] - m[j]) * di;
        }
#pragma unroll
    for (int j = 0; j < NC; j++) part[ph][j][lane] = acc[j];
    __syncthreads();
    if (ph == 0 && w < W) {
        const double cnt = last - first + 1;
        for (int j = 0; j < n; j++) {
            double v = part[0][j][lane];
            for (int p = 1; p < HS_PH; p++) v += part[p][j][lane];
            covs[(size_t)w * n * n + (size_t)i * n + j] = v / cnt;
        }
    }
}

// Per-GPU partial sums of the chain moments for the convergence exchange
// (TMpiChainCollector_UpdateCovAndCheckConverge, SampleCollector.f90:233-286):
// every walker is one chain with count = last-first+1 samples.
//   gmean == nullptr : out = [S0 = sum count, sum count*m (n), sum count*cov (n*n),
//                             sum cov (n*n), number of chains]
//   gmean != nullptr : out = sum count*(m-gmean)(m-gmean)^T (n*n)
// One block; each thread owns a fixed strided set of walkers and the partials
// are combined in a fixed tree order, so the sums are deterministic.
__global__ __launch_bounds__(256) void chain_moments_kernel(const double *means, const double *covs, int W, int n,
                                                           double count, const int *wcount, const double *gmean,
                                                           double *out)
{   // wcount (may be null): each walker's own sample count (collector windows)
    __shared__ double red[256];
    const int nout = gmean ? n * n : 2 + n + 2 * n * n;
    for (int o = 0; o < nout; o++) {
        double acc = 0.0;
        for (int w = threadIdx.x; w < W; w += 256) {
            const double *m = means + (size_t)w * n;
            const double *C = covs + (size_t)w * n * n;
            const double cw = wcount ? (double)wcount[w] : count;
            double v;
            if (gmean) {
                const int i = o / n, j = o % n;
                v = cw * (m[i] - gmean[i]) * (m[j] - gmean[j]);
            } else if (o == 0) {
                v = cw;
            } else if (o <= n) {
                v = cw * m[o - 1];
            } else if (o <= n + n * n) {
                v = cw * C[o - 1 - n];
            } else if (o <= n + 2 * n * n) {
                v = C[o - 1 - n - n * n];
            } else {
                v = 1.0;
            }
            acc += v;
        }
        red[threadIdx.x] = acc;
        __syncthreads();
        for (int h = 128; h > 0; h >>= 1) {
            if ((int)threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
            __syncthreads();
        }
        if (threadIdx.x == 0) out[o] = red[0];
        __syncthreads();
    }
}

void chain_moments_launch(const double *means, const double *covs, int W, int n, double count, const int *wcount,
                          const double *gmean, double *out, hipStream_t stream) {
    hipLaunchKernelGGL(chain_moments_kernel, dim3(1), dim3(256), 0, stream, means, covs, W, n, count, wcount, gmean,
                       out);
    HIP_CHECK(hipGetLastError());
}

// ------------------------------------------------------------ host side

static size_t mh_lds_bytes(const cmbs *s) {
    const DevCfg &d = s->dc;
    const int nd_st = d.stage_R ? d.rows.ND : d.rows.ND - d.rows.RR;
    const int ni_st = d.stage_cyc ? d.rows.NI : d.rows.CYC;
    const int ntd = d.stage_cov ? d.tl.n_dbl : d.tl.covinv;
    return (size_t)(nd_st + MAXLIKE + d.max_blk + d.tq_rows + d.def_cap * (QF_GROUPS + 1)) * MB * 8 +
           (size_t)((ntd + 31) & ~31) * 8 +
           (size_t)(ni_st + (d.stage_cyc ? d.all_n : 0)) * MB * 4 + (size_t)((d.tl.n_int + 63) & ~63) * 4 +
           MB * 4 + (size_t)d.np * MB * 8 + 2 * MB * 4 + 64;
}

static void set_mh_lds(cmbs *s) {
    // The mh_kernel LDS image: everything staged when it fits the 160 KB of a
    // CU; otherwise, in this order, the rotation rows, the cyclic-index
    // permutations (+ RandIndices scratch), the test-Gaussian tables and the
    // multi-wave scratch rows stay in HBM and are read in place.
    DevCfg &d = s->dc;
    const size_t cap = 160 * 1024;
    // the rotation rows stay in HBM when they are many (128 or more) and
    // every rotation wider than one parameter is drawn by rot_kernel: the
    // chain then only reads one column
    // per proposal (fetched beside the image, pre_blk), and staging the n x n
    // rows in and out of LDS is most of the image (config4_fast21: 441 of
    // ~600 rows)
    bool all_deferred = d.rot_defer != 0 && s->R_total >= 128;
    for (int bn : s->blk_n) all_deferred = all_deferred && (bn == 1 || bn >= ROT_DEFER_MIN);
    d.stage_R = s->stage_R_force >= 0 ? s->stage_R_force : (all_deferred ? 0 : 1);
    d.stage_cyc = d.stage_cov = 1;
    d.tq_rows = d.test_like ? 2 * s->n_used : 2;   // two per test-Gaussian row, or the proposal's block and step
    d.def_cap = (int)s->defer_likes.size();
    if (mh_lds_bytes(s) > cap) {               // the deferred combines go first: the likelihoods combine in-launch
        d.def_cap = 0;
        s->defer_likes.clear();
    }
    if (mh_lds_bytes(s) > cap) d.stage_R = 0;
    if (mh_lds_bytes(s) > cap) d.stage_cyc = 0;
    if (mh_lds_bytes(s) > cap) d.stage_cov = 0;
    if (mh_lds_bytes(s) > cap) d.tq_rows = 0;
    s->mh_lds = mh_lds_bytes(s);
    if (s->mh_lds > cap) fail(CMBL_ERR_ARG, "sampler state too large for LDS (%zu bytes)", s->mh_lds);
    if (!d.stage_cyc && !s->itmp_g.p) {
        s->itmp_g.alloc((size_t)std::max(1, s->all_n) * d.ld * 4);
        d.itmp_g = s->itmp_g.as<int>();
    }
    const int lds = (int)s->mh_lds;
    HIP_CHECK(hipFuncSetAttribute((const void *)mh_kernel<true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    HIP_CHECK(hipFuncSetAttribute((const void *)mh_kernel<true, false>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    HIP_CHECK(hipFuncSetAttribute((const void *)mh_kernel<false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
}

static void upload_tables(cmbs *s) {
    HIP_CHECK(hipDeviceSynchronize());     // the old tables may be read by queued kernels
    // padded to whole 256-byte LDS-DMA pieces
    s->tab_i.alloc(((s->h_tab_i.size() + 63) / 64 + 1) * 256);
    s->tab_i.upload(s->h_tab_i.data(), s->h_tab_i.size() * 4);
    s->tab_d.alloc(((s->h_tab_d.size() + 31) / 32 + 1) * 256);
    s->tab_d.upload(s->h_tab_d.data(), s->h_tab_d.size() * 8);
    s->dc.tab_i = s->tab_i.as<int>();
    s->dc.tab_d = s->tab_d.as<double>();
}

void sampler_create(cmbs *s, const cmbs_config_t *cfg) {
    if (cfg->n_walkers <= 0 || cfg->num_params <= 0 || cfg->num_params > MAXP)
        fail(CMBL_ERR_ARG, "n_walkers > 0 and 0 < num_params <= %d required", MAXP);
    if (cfg->n_used <= 0 || cfg->n_used > cfg->num_params) fail(CMBL_ERR_ARG, "bad n_used");
    s->W = cfg->n_walkers;
    s->np = cfg->num_params;
    s->n_used = cfg->n_used;
    s->params_used.assign(cfg->params_used, cfg->params_used + cfg->n_used);
    for (int p : s->params_used)
        if (p < 1 || p > s->np) fail(CMBL_ERR_ARG, "params_used entry %d out of range", p);
    // BlockedProposer Init (propose.f90:151-208)
    std::vector<int> used_blocks;
    for (int b = 0; b < cfg->n_blocks; b++) {
        const int n = cfg->block_n[b];
        if (n > MAXBLK) fail(CMBL_ERR_ARG, "block of %d parameters exceeds %d", n, MAXBLK);
        if (n > 0) {
            s->all_n += n;
            if (b + 1 <= cfg->slow_block_max) s->slow_n += n;
            used_blocks.push_back(b);
        }
    }
    std::vector<int> boff(cfg->n_blocks + 1, 0);
    for (int b = 0; b < cfg->n_blocks; b++) boff[b + 1] = boff[b] + cfg->block_n[b];
    s->fast_n = s->all_n - s->slow_n;
    s->nblocks = (int)used_blocks.size();
    if (s->nblocks == 0) fail(CMBL_ERR_ARG, "no parameter blocks");
    s->indices.assign(s->all_n, 0);
    s->proposer_for_index.assign(s->all_n, 0);
    int ix = 1;
    for (int i = 0; i < s->nblocks; i++) {
        const int ub = used_blocks[i];
        s->blk_start.push_back(ix);
        s->blk_n.push_back(cfg->block_n[ub]);
        for (int k = 0; k < cfg->block_n[ub]; k++) {
            const int u = cfg->block_params[boff[ub] + k];
            if (u < 1 || u > s->n_used) fail(CMBL_ERR_ARG, "block parameter %d not a used index", u);
            s->indices[ix - 1 + k] = u;
            s->proposer_for_index[ix - 1 + k] = i + 1;
        }
        ix += cfg->block_n[ub];
    }
    for (int v : s->indices)
        if (v == 0) fail(CMBL_ERR_ARG, "DecomposeCovariance: not all used parameters blocked");
    for (int i = 0; i < s->nblocks; i++) {
        const int nc = s->all_n - s->blk_start[i] + 1;
        s->blk_nchanged.push_back(nc);
        s->blk_changed_off.push_back((int)s->changed.size());
        s->blk_map_off.push_back(s->map_total);
        s->blk_R_off.push_back(s->R_total);
        for (int k = 0; k < nc; k++) {
            const int u = s->indices[s->blk_start[i] - 1 + k];
            s->used_params_changed_all.push_back(u);
            s->changed.push_back(s->params_used[u - 1] - 1);
        }
        s->map_total += nc * s->blk_n[i];
        s->R_total += s->blk_n[i] * s->blk_n[i];
    }
    if (s->all_n > MAXP) fail(CMBL_ERR_ARG, "too many parameters");

    const int np = s->np, W = s->W, nb = s->nblocks;
    DevCfg &d = s->dc;
    d.W = W;
    d.np = np;
    d.n_used = s->n_used;
    d.nblocks = nb;
    d.slow_n = s->slow_n;
    d.fast_n = s->fast_n;
    d.all_n = s->all_n;
    d.oversample_fast = cfg->oversample_fast < 1 ? 1 : cfg->oversample_fast;
    d.propose_scale = cfg->propose_scale;
    d.temperature = cfg->temperature > 0 ? cfg->temperature : 1.0;
    d.R_total = s->R_total;
    d.max_blk = 1;
    for (int bn : s->blk_n) d.max_blk = std::max(d.max_blk, bn);
    d.rot_defer = d.max_blk >= ROT_DEFER_MIN ? 1 : 0;
    d.bin_on = 0;

    // ---- shared tables
    TabLayout &tl = d.tl;
    auto &vi = s->h_tab_i;
    auto &vd = s->h_tab_d;
    auto put_i = [&](int &off, const std::vector<int> &v) {
        off = (int)vi.size();
        vi.insert(vi.end(), v.begin(), v.end());
    };
    auto put_d = [&](int &off, const double *v, int n) {
        off = (int)vd.size();
        vd.insert(vd.end(), v, v + n);
    };
    put_i(tl.blk_n, s->blk_n);
    put_i(tl.blk_nchanged, s->blk_nchanged);
    put_i(tl.blk_changed_off, s->blk_changed_off);
    put_i(tl.blk_map_off, s->blk_map_off);
    put_i(tl.blk_R_off, s->blk_R_off);
    put_i(tl.changed, s->changed);
    put_i(tl.pfi, s->proposer_for_index);
    std::vector<int> pu0(s->n_used);
    for (int i = 0; i < s->n_used; i++) pu0[i] = s->params_used[i] - 1;
    put_i(tl.params_used, pu0);
    tl.n_int = (int)vi.size();
    std::vector<double> zeros(std::max(s->map_total, np), 0.0);
    put_d(tl.mapping, zeros.data(), s->map_total);
    put_d(tl.pmin, cfg->pmin, np);
    put_d(tl.pmax, cfg->pmax, np);
    std::vector<double> pm(np, 0.0), ps(np, 0.0);
    std::vector<char> varying(np, 0);
    for (int p : s->params_used) varying[p - 1] = 1;
    bool has_pri = false;
    if (cfg->prior_mean && cfg->prior_std) {
        for (int i = 0; i < np; i++) {
            // GetLogPriors gate, calclike.f90:119 (TBaseParameters_ReadPriors :175 reads no prior otherwise)
            if (!varying[i] && !cfg->include_fixed_parameter_priors) continue;
            pm[i] = cfg->prior_mean[i];
            ps[i] = cfg->prior_std[i];
            has_pri |= ps[i] != 0.0;
        }
    }
    put_d(tl.pmean, pm.data(), np);
    put_d(tl.pstd, ps.data(), np);
    const int nlin = cfg->n_lincomb > 0 ? cfg->n_lincomb : 0;
    if (nlin && (!cfg->lincomb_weights || !cfg->lincomb_mean || !cfg->lincomb_std))
        fail(CMBL_ERR_ARG, "n_lincomb > 0 needs lincomb_weights, lincomb_mean and lincomb_std");
    put_d(tl.lin_w, cfg->lincomb_weights, nlin * np);
    put_d(tl.lin_m, cfg->lincomb_mean, nlin);
    put_d(tl.lin_s, cfg->lincomb_std, nlin);
    for (int k = 0; k < nlin; k++) has_pri |= cfg->lincomb_std[k] != 0.0;
    d.n_lin = nlin;
    tl.covinv = tl.center = (int)vd.size();   // set by cmbs_set_test_gaussian
    tl.n_dbl = (int)vd.size();
    d.has_priors = has_pri;
    d.test_like = 0;
    upload_tables(s);

    // ---- per-walker state rows
    Rows &R = d.rows;
    R.RR = (s->R_total + 1) & ~1;
    R.P = R.R + R.RR;
    R.T = R.P + np;
    R.L = R.T + np;
    R.M = R.L + 1;
    R.ND = (R.M + 2) & ~1;
    R.ACCF = R.BLKLP + nb;
    R.PROT = R.ACCF + 1;
    R.CYC = (R.PROT + 1 + 3) & ~3;
    R.NI = (R.CYC + s->all_n + s->slow_n + s->fast_n + 3) & ~3;
    d.ld = (W + NB - 1) / NB * NB;
    s->sd.alloc((size_t)R.ND * d.ld * 8);
    s->si.alloc((size_t)R.NI * d.ld * 4);
    HIP_CHECK(hipMemset(s->sd.p, 0, (size_t)R.ND * d.ld * 8));
    HIP_CHECK(hipMemset(s->si.p, 0, (size_t)R.NI * d.ld * 4));
    d.sd = s->sd.as<double>();
    d.si = s->si.as<int>();
    // rotation lists: walker indices [ld] + two counters per 64-walker range
    s->rot.alloc((size_t)(d.ld + 2 * (d.ld / 64)) * 4);
    HIP_CHECK(hipMemset(s->rot.p, 0, (size_t)(d.ld + 2 * (d.ld / 64)) * 4));
    d.rot_list = s->rot.as<int>();
    d.rot_cnt = d.rot_list + d.ld;
    s->rot_par.assign(d.ld / 64, 0);
    s->rot_lp.assign(d.ld / 64, 0);                   // every loop index starts at 0
    {   // the fast blocks: any deferred?  a single one (its width)?
        std::vector<int> fb;
        for (int q = s->slow_n; q < s->all_n; q++) {
            const int b = s->proposer_for_index[q] - 1;
            if (std::find(fb.begin(), fb.end(), b) == fb.end()) fb.push_back(b);
        }
        s->rot_fast_any = false;
        for (int b : fb) s->rot_fast_any = s->rot_fast_any || s->blk_n[b] >= ROT_DEFER_MIN;
        s->rot_fast_n = (fb.size() == 1 && s->blk_n[fb[0]] >= ROT_DEFER_MIN) ? s->blk_n[fb[0]] : 0;
        d.pre_blk = (fb.size() == 1 && s->blk_n[fb[0]] >= 2) ? fb[0] : -1;
        d.pre_off = d.pre_blk >= 0 ? s->blk_R_off[d.pre_blk] : 0;
        d.pre_n = d.pre_blk >= 0 ? s->blk_n[d.pre_blk] : 0;
        d.pre_lp = -1;
    }
    HIP_CHECK(hipFuncSetAttribute((const void *)rot_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)(ROT_WAVES * sizeof(RotLds))));

    set_mh_lds(s);

    // seeds
    std::vector<int> ij(W), kl(W);
    for (int w = 0; w < W; w++) cmbs_walker_seed(cfg->seed_ij, cfg->seed_kl, cfg->first_walker + w, &ij[w], &kl[w]);
    DevBuf dij(W * 4), dkl(W * 4);
    dij.upload(ij.data(), W * 4);
    dkl.upload(kl.data(), W * 4);
    hipLaunchKernelGGL(rng_init_kernel, dim3((W + 255) / 256), dim3(256), 0, 0, d, dij.as<int>(), dkl.as<int>());
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipDeviceSynchronize());
}

static void cholesky_lower(std::vector<double> &A, int n) {
    for (int j = 0; j < n; j++) {
        double dd = A[j * n + j];
        for (int k = 0; k < j; k++) dd -= A[j * n + k] * A[j * n + k];
        if (!(dd > 0.0)) fail(CMBL_ERR_NUMERIC, "Matrix_Cholesky: not positive definite %d", j + 1);
        dd = std::sqrt(dd);
        A[j * n + j] = dd;
        for (int i = j + 1; i < n; i++) {
            double x = A[i * n + j];
            for (int k = 0; k < j; k++) x -= A[i * n + k] * A[j * n + k];
            A[i * n + j] = x / dd;
        }
    }
    for (int i = 0; i < n; i++)
        for (int j = i + 1; j < n; j++) A[i * n + j] = 0.0;
}

void sampler_set_covariance(cmbs *s, const double *cov) {
    // BlockedProposer_SetCovariance, propose.f90:210-244 (host, once per update)
    const int n = s->n_used, na = s->all_n;
    std::vector<double> sig(n), corr((size_t)n * n);
    for (int i = 0; i < n; i++) {
        if (!(cov[i * n + i] > 0)) fail(CMBL_ERR_NUMERIC, "proposal covariance has non-positive diagonal");
        sig[i] = std::sqrt(cov[i * n + i]);
        for (int j = 0; j < n; j++) corr[i * n + j] = cov[i * n + j] / sig[i];
    }
    for (int i = 0; i < n; i++)
        for (int k = 0; k < n; k++) corr[k * n + i] = corr[k * n + i] / sig[i];
    std::vector<double> L((size_t)na * na);
    for (int i = 0; i < na; i++)
        for (int j = 0; j < na; j++) L[i * na + j] = corr[(s->indices[i] - 1) * n + (s->indices[j] - 1)];
    cholesky_lower(L, na);
    int uoff = 0;
    for (int i = 0; i < s->nblocks; i++) {
        const int bn = s->blk_n[i], st = s->blk_start[i], nc = s->blk_nchanged[i];
        for (int j = 0; j < nc; j++)
            for (int k = 0; k < bn; k++)
                s->h_tab_d[s->dc.tl.mapping + s->blk_map_off[i] + j * bn + k] =
                    sig[s->used_params_changed_all[uoff + j] - 1] * L[(st - 1 + j) * na + (st - 1 + k)];
        uoff += nc;
    }
    upload_tables(s);
}

void sampler_set_test_gaussian(cmbs *s, const double *cov, const double *center) {
    const int n = s->n_used;
    std::vector<double> A(cov, cov + (size_t)n * n);
    // Matrix_Inverse (test_likelihood inverts its covariance, calclike.f90:187-195)
    for (int i = 0; i < n; i++)
        if (std::fabs(A[i * n + i]) < 1e-30) fail(CMBL_ERR_NUMERIC, "Matrix_Inverse: very small diagonal");
    cholesky_lower(A, n);
    for (int j = 0; j < n; j++) {
        A[j * n + j] = 1.0 / A[j * n + j];
        for (int i = j + 1; i < n; i++) {
            double x = 0.0;
            for (int k = j; k < i; k++) x += A[i * n + k] * A[k * n + j];
            A[i * n + j] = -x / A[i * n + i];
        }
    }
    std::vector<double> T((size_t)n * n);
    for (int i = 0; i < n; i++)
        for (int j = 0; j <= i; j++) {
            double x = 0.0;
            for (int k = i; k < n; k++) x += A[k * n + i] * A[k * n + j];
            T[i * n + j] = T[j * n + i] = x;
        }
    auto &vd = s->h_tab_d;
    TabLayout &tl = s->dc.tl;
    vd.resize(tl.covinv);                   // replace any previous test_likelihood
    vd.insert(vd.end(), T.begin(), T.end());
    tl.center = (int)vd.size();
    vd.insert(vd.end(), center, center + s->np);
    tl.n_dbl = (int)vd.size();
    s->dc.test_like = 1;
    set_mh_lds(s);
    upload_tables(s);
}

static void set_change_mask(cmbs *s);

// Segment starts (absolute l, even) about TP_MAXL apart over [lo, hi] at which
// none of the bins [b.first, b.second] is split.
static std::vector<int> bin_safe_cuts(const std::vector<std::pair<int, int>> &bins, int lo, int hi, int L) {
    auto valid = [&](int c) {
        if (c % 2 != 0) return false;
        for (auto &b : bins)
            if (b.first < c && c <= b.second) return false;
        return true;
    };
    std::vector<int> cuts;
    int pos = lo;
    while (pos + L <= hi) {
        int c = -1;
        for (int x = pos + L; x > pos && c < 0; x--)
            if (valid(x)) c = x;
        for (int x = pos + L + 1; x <= hi && c < 0; x++)
            if (valid(x)) c = x;
        if (c < 0) break;
        cuts.push_back(c);
        pos = c;
    }
    return cuts;
}

// Fused window pass: a plik_lite likelihood (window stage kind 1) and a
// CMBlikes likelihood (kind 0) evaluated densely on the same theory buffer.
// The CMBlikes windows are re-segmented at l where no plik bin is split, so
// every column of both lies in one work item of the pass.
static void setup_fusion(cmbs *s) {
    s->tpass.reset();
    s->tp_like[0] = s->tp_like[1] = -1;
    s->pipe_ready = 0;
    s->tail_ready = 0;
    const int nl = (int)s->likes.size();
    auto sparse = [&](int i) {
        for (int q : s->sparse_likes)
            if (q == i) return true;
        return false;
    };
    s->tp_why = 0;
    for (int i = 0; i < nl; i++)
        for (int j = 0; j < nl; j++) {
            if (i == j) continue;
            s->tp_why = std::max(s->tp_why, 1);
            if (sparse(i) || sparse(j)) continue;
            const LikeSlot &P = s->likes[i], &C = s->likes[j];
            s->tp_why = std::max(s->tp_why, 2);
            if (P.dl != C.dl || P.ld_field != C.ld_field || P.ld_walker != C.ld_walker) continue;
            WinStage sp, sc;
            s->tp_why = std::max(s->tp_why, 3);
            if (!P.like->like->window_stage(sp) || sp.kind != 1) continue;
            s->tp_why = std::max(s->tp_why, 4);
            if (!C.like->like->window_stage(sc) || sc.kind != 0) continue;
            s->tp_why = std::max(s->tp_why, 5);
            std::map<int, std::vector<std::pair<int, int>>> bins;
            for (auto &c : sp.cols) bins[c.field].push_back({c.lo, c.hi});
            std::map<int, std::vector<int>> starts;
            for (auto &kv : bins) {
                int lo = 1 << 30, hi = -1;
                for (auto &c : sc.cols)
                    if (c.field == kv.first) {
                        lo = std::min(lo, c.lo);
                        hi = std::max(hi, c.hi);
                    }
                if (hi < lo) continue;
                starts[kv.first] = bin_safe_cuts(kv.second, lo & ~1, hi, TP_MAXL);
            }
            // the handle may be shared (standalone calls, other samplers): its
            // segmentation changes only if the fused pass is kept
            const auto saved = C.like->like->window_segments();
            if (!C.like->like->window_resegment(starts) || !C.like->like->window_stage(sc)) {
                C.like->like->window_set_segments(saved);
                continue;
            }
            s->tp_why = std::max(s->tp_why, 6);
            std::unique_ptr<TheoryPass> tp(new TheoryPass());
            if (!tp->build({sp, sc})) {
                C.like->like->window_set_segments(saved);
                continue;
            }
            s->tpass = std::move(tp);
            s->tp_like[0] = i;
            s->tp_like[1] = j;
            s->tp_stage[0] = sp;
            s->tp_stage[1] = sc;
            for (int k : s->tp_like) s->like_ws[k].release();
            size_t maxws = 0;   // the CMBlikes workspace follows its partial rows
            for (auto &l : s->likes) maxws = std::max(maxws, l.like->like->workspace_size(s->W));
            if (maxws > s->ws.bytes) s->ws.alloc(maxws);
            return;
        }
}

void sampler_add_likelihood(cmbs *s, cmbl_t *like, const int *nuisance_indices, const double *dl, long long ld_field,
                            long long ld_walker) {
    if (!like) fail(CMBL_ERR_ARG, "null likelihood");
    const int nn = like->like->n_nuis;
    if (nn > 0 && !nuisance_indices) fail(CMBL_ERR_ARG, "likelihood has %d nuisance parameters: indices needed", nn);
    std::vector<int> nidx(nn);
    for (int q = 0; q < nn; q++) {
        if (nuisance_indices[q] < 1 || nuisance_indices[q] > s->np)
            fail(CMBL_ERR_ARG, "nuisance index %d out of range 1..%d", nuisance_indices[q], s->np);
        nidx[q] = nuisance_indices[q] - 1;
    }
    if ((int)s->likes.size() >= MAXLIKE) fail(CMBL_ERR_ARG, "at most %d likelihoods per sampler", MAXLIKE);
    const int li = (int)s->likes.size();
    s->likes.push_back({like, nidx, dl, ld_field, ld_walker});
    // the index list joins the int table (LDS-staged with the proposer tables)
    s->dc.like_nidx[li] = (int)s->h_tab_i.size();
    s->h_tab_i.insert(s->h_tab_i.end(), nidx.begin(), nidx.end());
    s->dc.tl.n_int = (int)s->h_tab_i.size();
    set_mh_lds(s);
    upload_tables(s);
    const size_t nlk = (s->likes.size() + 1) & ~size_t(1);
    DevBuf nt(nlk * (size_t)s->dc.ld * 8);
    HIP_CHECK(hipMemset(nt.p, 0, nt.bytes));
    if (li > 0) HIP_CHECK(hipMemcpy(nt.p, s->like_terms.p, (size_t)li * s->dc.ld * 8, hipMemcpyDeviceToDevice));
    std::swap(nt.p, s->like_terms.p);
    std::swap(nt.bytes, s->like_terms.bytes);
    s->dc.n_like = (int)s->likes.size();
    s->dc.like_terms = s->like_terms.as<double>();
    {   // current-point terms: one more row, the existing ones kept
        DevBuf ct((size_t)s->likes.size() * s->dc.ld * 8);
        HIP_CHECK(hipMemset(ct.p, 0, ct.bytes));
        if (li > 0) HIP_CHECK(hipMemcpy(ct.p, s->cur_terms.p, (size_t)li * s->dc.ld * 8, hipMemcpyDeviceToDevice));
        std::swap(ct.p, s->cur_terms.p);
        std::swap(ct.bytes, s->cur_terms.bytes);
        s->dc.cur_terms = s->cur_terms.as<double>();
    }
    if (s->hist_cap > 0) {   // the terms ring follows the number of likelihoods
        s->hist_terms.alloc((size_t)s->hist_cap * s->likes.size() * s->W * 8);
        HIP_CHECK(hipMemset(s->hist_terms.p, 0, s->hist_terms.bytes));
    }
    s->nuis_bufs[li].alloc((size_t)std::max(nn, 1) * s->W * 8);
    s->dc.like_nuis[li] = s->nuis_bufs[li].as<double>();
    s->dc.like_nn[li] = nn;
    size_t maxws = 0;
    for (auto &l : s->likes) maxws = std::max(maxws, l.like->like->workspace_size(s->W));
    s->ws.alloc(maxws);
    set_change_mask(s);
    // likelihoods whose quadratic-form combine the accepting mh_kernel can take
    // over (dense evaluation only: the sparse ones write compacted slots)
    s->defer_likes.clear();
    for (int i = 0; i < (int)s->likes.size() && (int)s->defer_likes.size() < MAXDEF; i++) {
        bool sparse = false;
        for (int q : s->sparse_likes) sparse |= q == i;
        if (!sparse && s->likes[i].like->like->deferred_capable()) s->defer_likes.push_back(i);
    }
    for (int i = 0; i < MAXLIKE; i++) s->like_ws[i].release();
    set_mh_lds(s);
    setup_fusion(s);
    for (int i : s->defer_likes) s->like_ws[i].alloc(s->likes[i].like->like->workspace_size(s->W));
    for (int i : s->tp_like)
        if (i >= 0 && !s->like_ws[i].p) s->like_ws[i].alloc(s->likes[i].like->like->workspace_size(s->W));
    if (s->n_groups > 1) sampler_set_groups(s, s->n_groups);   // resize the group workspaces
}

// Change mask set-up (recomputed as likelihoods are added).  dependent_params
// of a CMB likelihood are its nuisance parameters (GeneralTypes.f90:648) and
// every theory parameter (CosmologyTypes.f90:154); here the theory parameters
// are the ones no likelihood owns as a nuisance parameter.  A likelihood whose
// dependent set misses some varying parameter can be skipped for walkers that
// did not move it; those that support it are evaluated on compacted walker
// slots (sparse), the others densely with the same keep-the-current-term rule.
static void set_change_mask(cmbs *s) {
    const int nl = (int)s->likes.size(), W = s->W;
    const size_t ld = s->dc.ld;
    unsigned long long nuis_all = 0;
    for (auto &l : s->likes)
        for (int i : l.nidx) nuis_all |= 1ull << i;
    const unsigned long long all = (s->np >= 64) ? ~0ull : ((1ull << s->np) - 1);
    const unsigned long long theory = all & ~nuis_all;
    s->sparse_likes.clear();
    for (int li = 0; li < nl; li++) {
        unsigned long long dep = theory;
        for (int i : s->likes[li].nidx) dep |= 1ull << i;
        s->dc.like_dep[li] = dep;
        bool maskable = false;
        for (int u : s->params_used) maskable |= !((dep >> (u - 1)) & 1ull);
        s->dc.like_out[li] = nullptr;
        if (maskable && s->likes[li].like->like->sparse_capable()) s->sparse_likes.push_back(li);
    }
    s->mask_on = !s->sparse_likes.empty();
    if (!s->mask_on) return;
    s->like_flag.alloc((size_t)nl * ld * 4);
    s->dc.like_flag = s->like_flag.as<int>();
    s->like_cnt.alloc(256);
    for (int li : s->sparse_likes) {
        const int nn = std::max(1, s->likes[li].like->like->n_nuis);
        s->like_outc[li].alloc((size_t)W * 8);
        s->like_nuisc[li].alloc((size_t)W * nn * 8 + (size_t)ld * 4);   // + the slot -> walker map
        s->dc.like_out[li] = s->like_outc[li].as<double>();
        if (s->likes[li].ld_walker != 0) s->like_dlc[li].alloc((size_t)W * s->likes[li].ld_walker * 8);
    }
}

// the likelihoods of a masked step: compaction of the sparse likelihoods'
// changed walkers, then every likelihood (sparse ones on the compacted slots)
// a deferrable likelihood's evaluation for the accepting mh_kernel that follows:
// the launches up to the quadratic form's partials, recorded in s->dc.def_*
static bool is_deferred(const cmbs *s, size_t i) {
    for (int q : s->defer_likes)
        if (q == (int)i) return true;
    return false;
}

static void record_deferred(cmbs *s, size_t i, const QFDeferred &d) {
    const int p = s->pending_def++;
    s->dc.def_like[p] = (int)i;
    s->dc.def_items[p] = d.n_items;
    s->dc.def_part[p] = d.partial;
    s->dc.def_add[p] = d.addend;
}

// the fused window pass over the whole walker set (eval_likes_fused)
static bool fused(const cmbs *s, size_t i) {
    return s->tpass && ((int)i == s->tp_like[0] || (int)i == s->tp_like[1]);
}

// the pass over theory rows dl (the walkers' own, or the drag's end points)
// with nuisance slices nuis[i] of likelihood i
static void launch_tpass(cmbs *s, hipStream_t stream, const double *dl, long long ld_field, long long ld_walker,
                         double *const *nuis) {
    TPOut o[2];
    for (int k = 0; k < 2; k++) {
        const int i = s->tp_like[k];
        const WinStage &st = s->tp_stage[k];
        Like &L = *s->likes[i].like->like;
        o[k] = TPOut{st.kind, st.cal_index, st.ld, 0, L.window_out(s->like_ws[i].p, s->W), st.X, nuis[i],
                     (long long)std::max(1, L.n_nuis)};
    }
    s->tpass->launch(dl, ld_field, ld_walker, o, s->W, stream);
}

static void launch_tpass(cmbs *s, hipStream_t stream) {
    const LikeSlot &P = s->likes[s->tp_like[0]];
    launch_tpass(s, stream, P.dl, P.ld_field, P.ld_walker, s->dc.like_nuis);
}

// The fused pass's two tails as one launch: when one fused likelihood is
// deferred and its quadratic form carries co-runs (plik_lite) and the other's
// whole after-window stage is a small chi^2 (Planck lensing), the chi^2's
// workgroups run in the quadratic form's launch (quadform_corun) and its term
// lands in its like_terms row as before.  The carrier and the carried index
// for this step, or -1, -1.
struct Corun {
    int carrier = -1, carried = -1;
    SmallGaussLaunch a{};
};

static Corun plan_corun(cmbs *s, bool defer) {
    Corun c;
    if (!defer || !s->tpass || s->no_corun) return c;
    for (int k = 0; k < 2; k++) {
        const int h = s->tp_like[k], o = s->tp_like[1 - k];
        Like &H = *s->likes[h].like->like;
        Like &O = *s->likes[o].like->like;
        if (!is_deferred(s, h) || !H.accepts_corun()) continue;
        if (O.corun_small(c.a, s->W, s->dc.like_nuis[o], O.n_nuis, s->like_terms.as<double>() + o * (size_t)s->dc.ld,
                          s->like_ws[o].p)) {
            c.carrier = h;
            c.carried = o;
            return c;
        }
    }
    return c;
}

// the rest of a fused likelihood after the pass: deferred or into its like_terms row
static void eval_after_window(cmbs *s, size_t i, bool defer, hipStream_t stream, const Corun &co) {
    if ((int)i == co.carried) return;   // inside the carrier's launch
    Like &L = *s->likes[i].like->like;
    const bool d = defer && is_deferred(s, i);
    const QFDeferred q = L.after_window(s->W, s->dc.like_nuis[i], L.n_nuis,
                                        d ? nullptr : s->like_terms.as<double>() + i * (size_t)s->dc.ld,
                                        s->like_ws[i].p, stream, d, (int)i == co.carrier ? &co.a : nullptr);
    if (d) record_deferred(s, i, q);
}

static bool eval_deferred(cmbs *s, size_t i, const double *nuis, hipStream_t stream) {
    if (!is_deferred(s, i)) return false;
    auto &l = s->likes[i];
    const QFDeferred d = l.like->like->loglike_batch_deferred(s->W, l.dl, l.ld_field, l.ld_walker, nuis,
                                                              l.like->like->n_nuis, s->like_ws[i].p, stream);
    record_deferred(s, i, d);
    return true;
}

static void eval_likes_masked(cmbs *s, hipStream_t stream, bool defer = false) {
    SparseSet ss{};
    const int ns = (int)s->sparse_likes.size();
    for (int b = 0; b < ns; b++) {
        const int li = s->sparse_likes[b];
        const int nn = s->likes[li].like->like->n_nuis;
        ss.like[b] = li;
        ss.nn[b] = nn;
        ss.nuisc[b] = s->like_nuisc[li].as<double>();
        ss.map[b] = reinterpret_cast<int *>(ss.nuisc[b] + (size_t)s->W * std::max(1, nn));
    }
    int *cnt = s->like_cnt.as<int>();
    hipLaunchKernelGGL(like_compact_kernel, dim3(ns), dim3(1024), 0, stream, s->dc, ss, cnt);
    HIP_CHECK(hipGetLastError());
    if (s->tpass) launch_tpass(s, stream);   // the fused likelihoods are dense (setup_fusion)
    const Corun co = plan_corun(s, defer);
    for (size_t i = 0; i < s->likes.size(); i++) {
        auto &l = s->likes[i];
        const int nn = l.like->like->n_nuis;
        int b = -1;
        for (int q = 0; q < ns; q++)
            if (ss.like[q] == (int)i) b = q;
        if (b < 0) {
            if (fused(s, i)) {
                eval_after_window(s, i, defer, stream, co);
                continue;
            }
            if (defer && eval_deferred(s, i, s->dc.like_nuis[i], stream)) continue;
            l.like->like->loglike_batch(s->W, l.dl, l.ld_field, l.ld_walker, s->dc.like_nuis[i], nn,
                                        s->like_terms.as<double>() + i * (size_t)s->dc.ld, s->ws.p, stream);
            continue;
        }
        const double *dl = l.dl;
        if (l.ld_walker != 0) {
            double *dlc = s->like_dlc[i].as<double>();
            hipLaunchKernelGGL(gather_theory_kernel, dim3(s->W), dim3(256), 0, stream, l.dl, l.ld_walker,
                               theory_extent(*l.like->like, l.ld_field), (const int *)ss.map[b], (const int *)(cnt + b),
                               dlc);
            HIP_CHECK(hipGetLastError());
            dl = dlc;
        }
        l.like->like->loglike_batch_sparse(s->W, dl, l.ld_field, l.ld_walker, ss.nuisc[b], nn,
                                           s->like_outc[i].as<double>(), s->ws.p, stream, cnt + b);
    }
}

// likelihood terms of walkers [g0, g1) at their trial points
// defer: the accepting mh_kernel launched next finishes the deferrable
// likelihoods (all walkers, one group)
static void eval_likes(cmbs *s, hipStream_t stream, bool gather, int g0, int g1, void *ws, bool defer = false) {
    const int Wg = g1 - g0;
    if (defer && (g0 != 0 || g1 != s->W)) fail(CMBL_ERR_ARG, "internal: deferred evaluation of a walker group");
    const size_t nl = s->likes.size();
    const bool fuse = s->tpass && g0 == 0 && g1 == s->W;
    if (fuse) {   // every nuisance slice first: the pass reads both likelihoods'
        if (gather)
            for (size_t i = 0; i < nl; i++) {
                const int nn = s->likes[i].like->like->n_nuis;
                hipLaunchKernelGGL(gather_nuis, dim3((s->W + 255) / 256), dim3(256), 0, stream,
                                   s->dc.sd + (size_t)s->dc.rows.T * s->dc.ld, s->W, s->dc.ld,
                                   s->dc.tab_i + s->dc.like_nidx[i], nn, s->dc.like_nuis[i]);
                HIP_CHECK(hipGetLastError());
            }
        gather = false;
        launch_tpass(s, stream);
    }
    const Corun co = fuse ? plan_corun(s, defer) : Corun{};
    // the likelihoods run in order on the caller's stream: side by side on forked
    // streams the memory-bound likelihood kernels slow each other more than they
    // overlap (MI355X, W = 1024, plik_lite + lensing: 77.1 vs 71.9 us/step; the
    // binning kernel alone 12.5 -> 26.2 us next to the lensing windows).  Even
    // the fused pass's two tails (quadratic form and the lensing chi^2, 13.6 and
    // 7.1 us) lose: with the chi^2 on a side stream forked and joined by events
    // the step took 87.5 instead of 63.3 us (round 2).  They share one launch
    // instead (plan_corun): 15.4 us against 13.5 + 4.6 (round 3)
    for (size_t i = 0; i < nl; i++) {
        hipStream_t st = stream;
        auto &l = s->likes[i];
        const int nn = l.like->like->n_nuis;
        double *nb = s->dc.like_nuis[i];
        if (gather) {   // mh_kernel scatters the nuisance slices itself on every step
            hipLaunchKernelGGL(gather_nuis, dim3((s->W + 255) / 256), dim3(256), 0, st,
                               s->dc.sd + (size_t)s->dc.rows.T * s->dc.ld, s->W, s->dc.ld,
                               s->dc.tab_i + s->dc.like_nidx[i], nn, nb);
            HIP_CHECK(hipGetLastError());
        }
        if (fuse && fused(s, i)) {
            eval_after_window(s, i, defer, st, co);
            continue;
        }
        if (defer && eval_deferred(s, i, nb, st)) continue;
        l.like->like->loglike_batch(Wg, l.dl + (size_t)g0 * l.ld_walker, l.ld_field, l.ld_walker,
                                    nb + (size_t)g0 * nn, nn, s->like_terms.as<double>() + i * (size_t)s->dc.ld + g0,
                                    ws, st);
    }
}

// the history ring slots of the next recorded step (none when history is off)
struct HistRow {
    double *p = nullptr;   // [n_used + 1][W]: used parameters, CurLike
    double *t = nullptr;   // [n_like][W]: per-likelihood terms
};

static HistRow next_hist(cmbs *s) {
    HistRow r;
    if (s->hist_cap == 0) return r;
    const size_t slot = (size_t)(s->hist_count % s->hist_cap);
    r.p = s->hist.as<double>() + slot * (s->n_used + 1) * s->W;
    if (!s->likes.empty() && s->hist_terms.p) r.t = s->hist_terms.as<double>() + slot * s->likes.size() * s->W;
    s->hist_count++;
    return r;
}

// Whether a proposing launch over the walker range from g0 can leave a
// rotation pending, so rot_kernel is worth launching.  Fast-only steps
// propose only fast blocks: none of them deferred, never.  With a single fast
// block every walker proposes in it at every fast-only step, so all of its
// loop indices move together and the host knows them (rot_lp: proposals so
// far mod n, or -1 once anything else has touched them: full steps, dragging,
// a loaded state, a new walker split); a rotation is due when it is 0 mod n.
static bool rot_may_pend(cmbs *s, int fast_only, int g0) {
    if (!s->dc.rot_defer) return false;
    int &lp = s->rot_lp[g0 / 64];
    if (!fast_only) {
        lp = -1;
        return true;
    }
    if (!s->rot_fast_any) return false;
    if (s->rot_fast_n == 0 || lp < 0) return true;
    const bool due = lp % s->rot_fast_n == 0;
    lp = (lp + 1) % s->rot_fast_n;
    return due;
}

static void rot_schedule_unknown(cmbs *s) { std::fill(s->rot_lp.begin(), s->rot_lp.end(), -1); }

// The in-launch hand-offs' give-up word (the unified launch, the bin co-run):
// a word of pinned host memory that the kernels write through its device
// mapping (pipe_giveup); zeroed here, checked once the step call's event has
// completed -- at the start of the next call and by the state readbacks
// (sampler_check_pipe) -- so a hand-off that gave up fails the run loudly
// instead of leaving silently rejected trials.
static void pipe_status_init(cmbs *s) {
    if (!s->pipe_status_host) {
        HIP_CHECK(hipHostMalloc((void **)&s->pipe_status_host, 64, hipHostMallocMapped | hipHostMallocCoherent));
        HIP_CHECK(hipHostGetDevicePointer((void **)&s->pipe_status_dev, s->pipe_status_host, 0));
        HIP_CHECK(hipEventCreateWithFlags(&s->pipe_ev, hipEventDisableTiming));
    }
    // no kernel of an earlier call still writes it: every call that launched a
    // hand-off kernel recorded pipe_ev after it (pipe_status_post, also on the
    // error paths), so waiting on this sampler's event suffices -- other
    // samplers' and the caller's work on the device are not waited for
    if (s->pipe_ev_pending) HIP_CHECK(hipEventSynchronize(s->pipe_ev));
    *reinterpret_cast<volatile int *>(s->pipe_status_host) = 0;
    s->pipe_ev_pending = false;
}

static void pipe_status_post(cmbs *s, hipStream_t stream) {
    HIP_CHECK(hipEventRecord(s->pipe_ev, stream));
    s->pipe_ev_pending = true;
}

// on an error path: the event covers whatever this call launched before it
static void pipe_status_post_nothrow(cmbs *s, hipStream_t stream) {
    if (s->pipe_ev && hipEventRecord(s->pipe_ev, stream) == hipSuccess) s->pipe_ev_pending = true;
}

void sampler_check_pipe(cmbs *s, bool wait) {
    if (!s->pipe_ev_pending) return;
    if (wait) HIP_CHECK(hipEventSynchronize(s->pipe_ev));
    const hipError_t q = hipEventQuery(s->pipe_ev);
    if (q == hipErrorNotReady) return;   // checked at a later call
    HIP_CHECK(q);
    s->pipe_ev_pending = false;
    if (*reinterpret_cast<volatile int *>(s->pipe_status_host) & CMBL_STATUS_PIPE_WAIT) {
        *reinterpret_cast<volatile int *>(s->pipe_status_host) = 0;
        s->tail_ready = 0;
        s->pipe_ready = 0;
        fail(CMBL_ERR_NUMERIC, "a pipelined step's in-launch hand-off gave up waiting (CMBL_STATUS_PIPE_WAIT): "
                               "the walkers' last steps are invalid");
    }
}

// Whether this run of fast steps can take the bin co-run: one likelihood,
// plik_lite, deferred (its quadratic form's combine in the next mh launch),
// no fused pass, one walker group, no change mask.  Allocates the raw sums and
// sets up the calibration hand-off (as pipe_setup).
static bool bin_setup(cmbs *s, int fast_only, PlikBinArgs &pb) {
    // (mode 3 needs the fused pass, so it falls back here with plik_lite alone)
    if (s->pipe_mode == 0 || !fast_only || s->tpass || s->n_groups != 1 || s->mask_on ||
        s->likes.size() != 1 || !is_deferred(s, 0))
        return false;
    const LikeSlot &L = s->likes[0];
    WinStage st;
    if (!L.like->like->bin_args(pb, L.dl, L.ld_field, L.ld_walker) || !L.like->like->window_stage(st) ||
        st.cal_index < 0)
        return false;
    const size_t need = (size_t)QuadForm::wpad(s->W) * pb.Np * 8;
    if (s->bin_S.bytes < need) {
        s->bin_S.alloc(need);
        HIP_CHECK(hipMemset(s->bin_S.p, 0, need));
    }
    for (int f = 0; f < 3; f++)
        if (pb.fr.b1[f] - pb.fr.b0[f] > 2 * MH_THREADS) return false;   // mh_bin_kernel: two bins a thread
    s->bin_lds = std::max(s->mh_lds, (size_t)pb.lds_doubles * 8);
    if (s->bin_lds > 160 * 1024) return false;
    HIP_CHECK(hipFuncSetAttribute((const void *)mh_bin_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)s->bin_lds));
    HIP_CHECK(hipFuncSetAttribute((const void *)mh_bin_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)s->bin_lds));
    if (s->pipe_ready == s->W) return true;
    pipe_status_init(s);
    {   // both halves unset: the first launch publishes into half 1, resets half 0
        const std::vector<unsigned long long> unset((size_t)4 * s->dc.ld, TP_PIPE_UNSET);
        s->pipe_cal.alloc(unset.size() * 8);
        s->pipe_cal.upload(unset.data(), unset.size() * 8);
    }
    s->pipe_epoch = 0;
    s->pipe_ready = s->W;
    return true;
}

// plik's deferred quadratic form over the Delta rows the bin co-run (and
// rot_kernel) formed; its combine runs in the next Metropolis launch
static void launch_bin_qf(cmbs *s, hipStream_t stream) {
    Like &Q = *s->likes[0].like->like;
    const QFDeferred d = Q.after_window(s->W, s->dc.like_nuis[0], std::max(1, Q.n_nuis), nullptr, s->like_ws[0].p,
                                        stream, true);
    record_deferred(s, 0, d);
}

// The lean chain's LDS (mhlean.h's carve)
static size_t lean_lds_bytes(const cmbs *s) {
    const Rows &R = s->dc.rows;
    return (size_t)(R.R + R.ND - R.P + MAXDEF * (QF_GROUPS + 1) + s->np) * MB * 8 + (size_t)(8 + 3) * MB * 4;
}

// Whether a launch of fast-only steps takes the lean chain (mhlean.h): the
// only fast parameter is a one-parameter block, no test likelihood, no
// linear-combination priors, no change mask; and that block's constants.
static LeanCfg lean_cfg(const cmbs *s, int fast_only, bool masked) {
    LeanCfg L{};
    const DevCfg &d = s->dc;
    if (s->lean_off || !fast_only || masked || s->fast_n != 1 || d.test_like || d.n_lin || d.n_like > MAXLIKE)
        return L;
    const int b = s->proposer_for_index[s->slow_n] - 1;
    if (s->blk_n[b] != 1 || s->blk_nchanged[b] > LEAN_MAXC || lean_lds_bytes(s) > s->mh_lds) return L;
    for (int l = 0; l < d.n_like; l++) {
        const std::vector<int> &ni = s->likes[l].nidx;
        if ((int)ni.size() > LEAN_MAXQ) return LeanCfg{};
        L.nn[l] = (int)ni.size();
        for (size_t q = 0; q < ni.size(); q++) L.nuis[l][q] = ni[q];
    }
    L.nc = s->blk_nchanged[b];
    for (int j = 0; j < L.nc; j++) {
        L.chg[j] = s->changed[s->blk_changed_off[b] + j];
        L.map[j] = s->h_tab_d[d.tl.mapping + s->blk_map_off[b] + j];
    }
    L.r_row = d.rows.R + s->blk_R_off[b];
    L.cyc_row = d.rows.CYC + s->all_n + s->slow_n;
    L.blklp_row = d.rows.BLKLP + b;
    L.on = 1;
    return L;
}

static void launch_mh(cmbs *s, bool accept, bool propose, int fast_only, const HistRow &row, hipStream_t stream,
                      int g0, int g1, bool masked = false, const PlikBinArgs *bin = nullptr) {
    const dim3 g((g1 - g0 + MB - 1) / MB), b(MH_THREADS);
    const int blk0 = g0 / MB;
    const size_t lds = s->mh_lds;
    DevCfg dc = s->dc;
    dc.mask_on = masked ? 1 : 0;
    dc.lean = lean_cfg(s, fast_only, masked);
    if (s->pending_def && !accept) fail(CMBL_ERR_ARG, "internal: deferred likelihoods without an accepting step");
    dc.pre_lp = -1;   // the single deferred block's loop index before this launch's proposals (rot_may_pend)
    if (propose && fast_only && s->dc.rot_defer && s->rot_fast_n > 0 && dc.pre_blk >= 0 && s->rot_lp[g0 / 64] >= 0)
        dc.pre_lp = s->rot_lp[g0 / 64];
    const bool rot = propose && rot_may_pend(s, fast_only, g0);
    if (rot) {                       // alternate the two rotation-list counters of this walker range
        dc.rot_par = s->rot_par[g0 / 64];
        s->rot_par[g0 / 64] ^= 1;
    }
    dc.n_def = s->pending_def;
    s->pending_def = 0;
    dc.pub_on = 0;
    if (bin) {   // mh_bin_kernel: the proposing launch bins the theory beside the Metropolis workgroups
        if (!propose || g0 != 0 || g1 != s->W) fail(CMBL_ERR_ARG, "internal: bin co-run launch");
        Like &Q = *s->likes[0].like->like;
        WinStage st;
        Q.window_stage(st);
        dc.pub_on = s->tail_nosignal ? 0 : 1;   // debug: never publish (the give-up test)
        dc.pub_pcal[0] = s->likes[0].nidx[st.cal_index];
        dc.pub_pcal[1] = -1;
        const unsigned e = s->pipe_epoch + 1;   // this launch's half e % 2; it resets the other for the next
        dc.calbuf = s->pipe_cal.as<double>() + (size_t)(e % 2) * 2 * dc.ld;
        dc.calbuf_next = s->pipe_cal.as<double>() + (size_t)((e + 1) % 2) * 2 * dc.ld;
        dc.bin_on = 1;
        dc.bin_nused = bin->nused;
        dc.bin_Np = bin->Np;
        dc.bin_cal = st.cal_index;
        dc.bin_S = s->bin_S.as<double>();
        dc.bin_X = bin->X;
        dc.bin_delta = Q.window_out(s->like_ws[0].p, s->W);
        const int nmh = (int)g.x, nmh_pad = (nmh + 7) / 8 * 8;
        const dim3 gb(nmh_pad + s->W);
        try {
            timed_launch("mh_bin_kernel", stream, [&](hipEvent_t e0, hipEvent_t e1) {
                if (accept)
                    hipExtLaunchKernelGGL(mh_bin_kernel<true>, gb, b, s->bin_lds, stream, e0, e1, 0, dc, fast_only,
                                          row.p, row.t, nmh, nmh_pad, *bin, s->pipe_status_dev);
                else
                    hipExtLaunchKernelGGL(mh_bin_kernel<false>, gb, b, s->bin_lds, stream, e0, e1, 0, dc, fast_only,
                                          row.p, row.t, nmh, nmh_pad, *bin, s->pipe_status_dev);
            });
            HIP_CHECK(hipGetLastError());
        } catch (...) {
            s->pipe_ready = 0;   // both halves re-uploaded as unset next time
            pipe_status_post_nothrow(s, stream);
            throw;
        }
        s->pipe_epoch = e;
    } else
    timed_launch("mh_kernel", stream, [&](hipEvent_t e0, hipEvent_t e1) {
        if (accept && propose)
            hipExtLaunchKernelGGL(mh_kernel<true, true>, g, b, lds, stream, e0, e1, 0, dc, fast_only, row.p, row.t, blk0);
        else if (accept)
            hipExtLaunchKernelGGL(mh_kernel<true, false>, g, b, lds, stream, e0, e1, 0, dc, fast_only, row.p, row.t, blk0);
        else
            hipExtLaunchKernelGGL(mh_kernel<false, true>, g, b, lds, stream, e0, e1, 0, dc, fast_only, row.p, row.t, blk0);
    });
    if (rot) {                       // the walkers whose proposal waits on a new rotation
        HIP_CHECK(hipGetLastError());
        timed_launch("rot_kernel", stream, [&](hipEvent_t e0, hipEvent_t e1) {
            hipExtLaunchKernelGGL(rot_kernel, dim3((g1 - g0 + ROT_WAVES - 1) / ROT_WAVES), dim3(64 * ROT_WAVES),
                                  ROT_WAVES * sizeof(RotLds), stream, e0, e1, 0, dc, g0);
        });
    }
    HIP_CHECK(hipGetLastError());
}

void sampler_set_start(cmbs *s, const double *P0, hipStream_t stream) {
    // host [W][np] -> device trial rows [np][W]
    std::vector<double> t((size_t)s->np * s->W);
    for (int w = 0; w < s->W; w++)
        for (int i = 0; i < s->np; i++) t[(size_t)i * s->W + w] = P0[(size_t)w * s->np + i];
    HIP_CHECK(hipMemcpy2DAsync(s->dc.sd + (size_t)s->dc.rows.T * s->dc.ld, (size_t)s->dc.ld * 8, t.data(),
                               (size_t)s->W * 8, (size_t)s->W * 8, s->np, hipMemcpyHostToDevice, stream));
    // t is pageable and local: the copy must be complete before anything below can throw and unwind it
    HIP_CHECK(hipStreamSynchronize(stream));
    eval_likes(s, stream, true, 0, s->W, s->ws.p);
    hipLaunchKernelGGL(start_kernel, dim3((s->W + 255) / 256), dim3(256), 0, stream, s->dc);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipStreamSynchronize(stream));
    s->started = true;
}

static void check_theory_fresh(const cmbs *s) {
    if (s->theory_stale)
        fail(CMBL_ERR_ARG, "resumed from a state image whose walkers moved their slow parameters: recompute the "
                           "theory at the restored points with cmbs_refresh_theory before stepping");
}

// The unified pipelined fast steps (mh_step_kernel, steptail.h): whether this run of fast steps
// can take them -- the fused pass's vectorised form over one walker group, no
// change mask, no rotations left to rot_kernel, and its two stages a deferred
// quadratic form (plik_lite: every row calibrated) and a small chi^2 another
// launch can carry (Planck lensing).  Sets up the raw-sum buffers once per W.
static bool tail_setup(cmbs *s, int fast_only) {
    // (the unified launch carries the fused pair alone: with a third likelihood the
    // run takes the unpipelined steps, whose eval_likes runs every likelihood; BASELINE
    // configs[2] with a lowl term would be such a run -- clik is absent, so none exists here)
    if (s->pipe_mode == 0 || !fast_only || !s->tpass || s->n_groups != 1 || s->mask_on ||
        (s->dc.rot_defer && s->rot_fast_any) || s->likes.size() != 2)
        return false;
    {
        const LikeSlot &P = s->likes[s->tp_like[0]];
        if (!s->tpass->vec_ok(P.dl, P.ld_field, P.ld_walker)) return false;
    }
    if (s->tail_ready == s->W) return true;
    if (s->tail_ready == -s->W) return false;
    s->tail_ready = -s->W;
    s->tail_qf = s->tail_g = -1;
    for (int k = 0; k < 2; k++) {
        const int i = s->tp_like[k];
        Like &L = *s->likes[i].like->like;
        const WinStage &st = s->tp_stage[k];
        QFSource src;
        if (st.kind == 1 && is_deferred(s, (size_t)i) && L.qf_source(src, s->W, s->like_ws[i].p)) {
            bool all_cal = st.cal_index >= 0;
            for (const WinCol &c : st.cols) all_cal = all_cal && c.cal;
            if (all_cal && st.ld == src.Np) s->tail_qf = k;
        }
        SmallGaussLaunch g{};
        if (st.kind == 0 && L.corun_small(g, s->W, s->dc.like_nuis[i], L.n_nuis,
                                          s->like_terms.as<double>() + (size_t)i * s->dc.ld, s->like_ws[i].p))
            s->tail_g = k;
    }
    if (s->tail_qf < 0 || s->tail_g < 0 || s->tail_qf == s->tail_g) return false;
    const size_t Wp = (size_t)QuadForm::wpad(s->W);
    int rows = 0;
    for (const WinCol &c : s->tp_stage[s->tail_g].cols) rows = std::max(rows, c.row + 1);
    const size_t bytes[2] = {Wp * (size_t)s->tp_stage[s->tail_qf].ld * 8, (size_t)rows * s->W * 8};
    for (int p = 0; p < 2; p++)
        for (int k = 0; k < 2; k++) {
            const size_t b = bytes[k == s->tail_qf ? 0 : 1];
            s->tail_S[p][k].alloc(b);
            HIP_CHECK(hipMemset(s->tail_S[p][k].p, 0, b));   // padding rows / columns stay 0
        }
    std::vector<unsigned char> rc((size_t)rows + 16, 0);
    for (const WinCol &c : s->tp_stage[s->tail_g].cols) rc[c.row] = c.cal ? 1 : 0;
    s->tail_rowcal.alloc(rc.size());
    s->tail_rowcal.upload(rc.data(), rc.size());
    // the unified launch's arrival counters (from 0, epoch 0) and its LDS
    s->tail_cnt_bytes = (Wp / QF_TILE * TW_PAD * 4 + 15) & ~(size_t)15;   // a multiple of 16 from the start
    s->tail_cnt.alloc(s->tail_cnt_bytes);
    HIP_CHECK(hipMemset(s->tail_cnt.p, 0, s->tail_cnt_bytes));
    s->tail_epoch = 0;
    s->tail_epoch_g = 0;
    pipe_status_init(s);
    {
        const int gi = s->tp_like[s->tail_g];
        Like &G = *s->likes[gi].like->like;
        SmallGaussLaunch g{};
        G.corun_small(g, s->W, s->dc.like_nuis[gi], G.n_nuis, s->like_terms.as<double>() + (size_t)gi * s->dc.ld,
                      s->like_ws[gi].p);
        s->uni_lds = std::max({s->mh_lds, (size_t)QFS_LDS_DOUBLES * 8, (size_t)tp_vec_lds_bytes<2>(),
                               (size_t)small_gauss_lds_doubles<UNI_WT>(g.d.nX) * 8,
                               (size_t)small_gauss_lds_doubles<MB>(g.d.nX) * 8});
        for (const void *k : {(const void *)mh_step_kernel<false, true>, (const void *)mh_step_kernel<true, true>,
                              (const void *)mh_step_kernel<true, false>, (const void *)mh_tail_kernel<true, true>,
                              (const void *)mh_tail_kernel<true, false>})
            HIP_CHECK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)s->uni_lds));
    }
    for (auto &pl : s->uni_plan) pl.key[0] = -1;
    s->tail_ready = s->W;
    return true;
}

// One step tail: the quadratic form and the chi^2 of the step whose raw sums
// are in half rd (rd < 0: none), and the pass storing the next step's raw sums
// into half wr (wr < 0: none).
static StepTail make_tail(cmbs *s, int rd, int wr) {
    StepTail t;
    const int W = s->W;
    t.W = W;
    if (rd >= 0) {
        const int qi = s->tp_like[s->tail_qf], gi = s->tp_like[s->tail_g];
        Like &Q = *s->likes[qi].like->like;
        Like &G = *s->likes[gi].like->like;
        if (!Q.qf_source(t.q.src, W, s->like_ws[qi].p)) fail(CMBL_ERR_ARG, "internal: step tail quadratic form");
        t.q.S = s->tail_S[rd][s->tail_qf].as<double>();
        t.q.nuis = s->dc.like_nuis[qi];
        t.q.ld_nuis = std::max(1, Q.n_nuis);
        t.q.cal_index = s->tp_stage[s->tail_qf].cal_index;
        t.q.W = W;
        t.nq = t.q.src.n_items * (QuadForm::wpad(W) / QF_TILE);
        if (!G.corun_small(t.g, W, s->dc.like_nuis[gi], G.n_nuis, s->like_terms.as<double>() + (size_t)gi * s->dc.ld,
                           s->like_ws[gi].p))
            fail(CMBL_ERR_ARG, "internal: step tail chi^2");
        t.g.partial = s->tail_S[rd][s->tail_g].as<double>();
        t.g.row_cal = s->tail_rowcal.as<unsigned char>();
        t.g.stage_cal = s->tp_stage[s->tail_g].cal_index;
        t.ng = (W + UNI_WT - 1) / UNI_WT;
        // the chi^2 folded into the Metropolis workgroups: bit-identical while its
        // 16-walker body's thread groups (256 / 16) cover the bandpowers
        // (middle launches only: in the accept-only launch that ends a call the
        // chi^2 would sit on the chain's critical path, 21.5 against 23.3 us)
        t.fold_g = (s->fold_g && wr >= 0 && t.g.d.nX <= MH_THREADS / MB) ? 1 : 0;
        t.qf_ahead = s->qf_ahead;
        t.qf_prio = s->qf_prio;
        t.fold_tpf = s->fold_tpf;
        t.fold_late_prio = s->fold_late_prio;
        if (t.fold_g) t.ng = 0;
    }
    if (wr >= 0) {
        TPOut o[2];
        for (int k = 0; k < 2; k++) {
            const int i = s->tp_like[k];
            const WinStage &st = s->tp_stage[k];
            Like &L = *s->likes[i].like->like;
            o[k] = TPOut{st.kind, st.cal_index, st.ld, 0, s->tail_S[wr][k].as<double>(), st.X, s->dc.like_nuis[i],
                         (long long)std::max(1, L.n_nuis)};
        }
        t.tp = s->tpass->dev_args(o, W);
        const LikeSlot &P = s->likes[s->tp_like[0]];
        t.dl = P.dl;
        t.ld_field = P.ld_field;
        t.ld_walker = P.ld_walker;
        t.np = s->tpass->n_blocks();
    }
    return t;
}

// One unified step launch (pipe_mode 3, mh_step_kernel): the tails of the
// step whose raw sums are in half rd (rd < 0: none), the pass into half wr
// (wr < 0: none), and the Metropolis workgroups accepting that step (when
// rd >= 0) and proposing the next (propose).
static void launch_unified(cmbs *s, hipStream_t stream, bool propose, int rd, int wr, const HistRow &row,
                           int fast_only) {
    const bool accept = rd >= 0;
    StepTail t = make_tail(s, rd, wr);
    DevCfg dc = s->dc;
    dc.mask_on = 0;
    dc.lean = lean_cfg(s, fast_only, false);
    dc.pub_on = 0;
    dc.n_def = 0;
    s->pending_def = 0;
    if (accept) {   // plik's combine from this launch's partials (QFDeferred)
        dc.n_def = 1;
        dc.def_like[0] = s->tp_like[s->tail_qf];
        dc.def_items[0] = t.q.src.n_items;
        dc.def_part[0] = t.q.src.partial;
        dc.def_add[0] = nullptr;
    }
    const int ng_rows = t.ng;
    TailWait tw{};
    tw.cnt = s->tail_cnt.as<unsigned int>();
    tw.epoch = s->tail_epoch + (accept ? 1u : 0u);
    tw.epoch_g = s->tail_epoch_g + ((accept && !t.fold_g) ? 1u : 0u);
    tw.nq_items = t.q.src.n_items;
    tw.ng = accept ? (s->W + UNI_WT - 1) / UNI_WT : 0;   // an unfolded launch's chi^2 workgroups (the target's
    tw.gwt = UNI_WT;                                      // per-tile count for the epoch_g launches)
    tw.status = s->pipe_status_dev;
    tw.nosignal = s->tail_nosignal;
    tw.stamp_slot = propose ? 0 : 1;
    tw.ntiles = (int)(s->tail_cnt_bytes / 4);
    const int nmh = (s->W + MB - 1) / MB;
    const int v = accept ? (propose ? 1 : 2) : 0;
    StepTailPlan &pl = s->uni_plan[v];
    if (pl.key[0] != t.nq || pl.key[1] != ng_rows || pl.key[2] != t.np) {
        const std::vector<int2> rows = tail_rows(t.nq, ng_rows, t.np, nmh);
        pl.d_rows.alloc(rows.size() * sizeof(int2));
        pl.d_rows.upload(rows.data(), rows.size() * sizeof(int2));
        pl.nrows = (int)rows.size();
        pl.key[0] = t.nq;
        pl.key[1] = ng_rows;
        pl.key[2] = t.np;
    }
    const dim3 grid((unsigned)pl.nrows * 8), b(MH_THREADS);
    const int2 *rows = pl.d_rows.as<int2>();
    static const char *names[3] = {"mh_step_first", "mh_step_kernel", "mh_step_last"};
    static const char *cnames[3] = {"mh_step_first", "mh_tail_kernel", "mh_tail_last"};
    const bool cached = s->binned_cache && accept && wr < 0 && rd == 0;   // the binned-cache steps (no pass)
    try {
        timed_launch(cached ? cnames[v] : names[v], stream, [&](hipEvent_t e0, hipEvent_t e1) {
            if (cached && v == 1)
                hipExtLaunchKernelGGL(mh_tail_kernel<true, true>, grid, b, s->uni_lds, stream, e0, e1, 0, dc,
                                      fast_only, row.p, row.t, t, rows, tw, nmh);
            else if (cached && v == 2)
                hipExtLaunchKernelGGL(mh_tail_kernel<true, false>, grid, b, s->uni_lds, stream, e0, e1, 0, dc,
                                      fast_only, row.p, row.t, t, rows, tw, nmh);
            else if (v == 0)
                hipExtLaunchKernelGGL(mh_step_kernel<false, true>, grid, b, s->uni_lds, stream, e0, e1, 0, dc,
                                      fast_only, row.p, row.t, t, rows, tw, nmh);
            else if (v == 1)
                hipExtLaunchKernelGGL(mh_step_kernel<true, true>, grid, b, s->uni_lds, stream, e0, e1, 0, dc, fast_only,
                                      row.p, row.t, t, rows, tw, nmh);
            else
                hipExtLaunchKernelGGL(mh_step_kernel<true, false>, grid, b, s->uni_lds, stream, e0, e1, 0, dc,
                                      fast_only, row.p, row.t, t, rows, tw, nmh);
        });
        HIP_CHECK(hipGetLastError());
    } catch (...) {
        s->tail_ready = 0;   // the counters and the epoch are set up afresh next time
        pipe_status_post_nothrow(s, stream);
        throw;
    }
    if (accept) s->tail_epoch++;
    if (accept && !t.fold_g) s->tail_epoch_g++;
}

void sampler_step(cmbs *s, int n_steps, int fast_only, hipStream_t stream) {
    if (!s->started) fail(CMBL_ERR_ARG, "cmbs_set_start must be called before cmbs_step");
    check_theory_fresh(s);
    if (fast_only && s->fast_n == 0) fail(CMBL_ERR_ARG, "no fast parameters");
    if (!fast_only && s->slow_n > 0 && !s->likes.empty())
        fail(CMBL_ERR_ARG, "slow proposals need the theory at the trial point: use cmbs_step_theory");
    if (n_steps <= 0) return;
    // propose(1) | likes | accept(1)+propose(2) | likes | ... | likes | accept(n)
    const int G = s->n_groups;
    sampler_check_pipe(s);
    if (G == 1 && tail_setup(s, fast_only)) {
        // unified: propose(1) + pass(1) | tails(1) + pass(2) + accept(1) + propose(2) | ... |
        // tails(n) + accept(n): one launch per step.  The arrival counters start from 0
        // in every call (the first launch zeroes them; the epochs are counted within it)
        s->tail_epoch = 0;
        s->tail_epoch_g = 0;
        launch_unified(s, stream, true, -1, 0, HistRow{}, fast_only);
        if (s->binned_cache) {
            // the theory is fixed within the call: every step's tails read the raw
            // sums the first launch's pass wrote (half 0), and no launch re-bins
            for (int k = 0; k < n_steps; k++)
                launch_unified(s, stream, k + 1 < n_steps, 0, -1, next_hist(s), fast_only);
        } else
        for (int k = 0; k < n_steps; k++)
            launch_unified(s, stream, k + 1 < n_steps, k % 2, k + 1 < n_steps ? (k + 1) % 2 : -1, next_hist(s),
                           fast_only);
        pipe_status_post(s, stream);
        return;
    }
    PlikBinArgs pb;
    if (G == 1 && bin_setup(s, fast_only, pb)) {
        // bin co-run: propose(1) + bins(1) | [rotations] | quadform(1) | accept(1) + propose(2) + bins(2) |
        // ... | quadform(n) | accept(n)
        for (int k = 0; k < n_steps; k++) {
            launch_mh(s, k > 0, true, fast_only, k > 0 ? next_hist(s) : HistRow{}, stream, 0, s->W, false, &pb);
            launch_bin_qf(s, stream);
        }
        launch_mh(s, true, false, fast_only, next_hist(s), stream, 0, s->W, false);
        pipe_status_post(s, stream);
        return;
    }
    if (G == 1) {
        const bool m = s->mask_on;
        launch_mh(s, false, true, fast_only, HistRow{}, stream, 0, s->W, m);
        if (m) eval_likes_masked(s, stream, true);
        else eval_likes(s, stream, false, 0, s->W, s->ws.p, true);
        for (int k = 1; k < n_steps; k++) {
            launch_mh(s, true, true, fast_only, next_hist(s), stream, 0, s->W, m);
            if (m) eval_likes_masked(s, stream, true);
            else eval_likes(s, stream, false, 0, s->W, s->ws.p, true);
        }
        launch_mh(s, true, false, fast_only, next_hist(s), stream, 0, s->W, m);
        return;
    }
    // groups are independent chains: fork from the caller's stream, issue the
    // step chain of every group breadth-first so the queues interleave, join
    HIP_CHECK(hipEventRecord(s->events[MAXGROUPS], stream));
    for (int g = 0; g < G; g++) HIP_CHECK(hipStreamWaitEvent(s->streams[g], s->events[MAXGROUPS], 0));
    for (int k = 0; k <= n_steps; k++) {
        const HistRow row = k > 0 ? next_hist(s) : HistRow{};
        for (int g = 0; g < G; g++) {
            const int g0 = s->grp0[g], g1 = s->grp0[g + 1];
            launch_mh(s, k > 0, k < n_steps, fast_only, row, s->streams[g], g0, g1);
            if (k < n_steps) eval_likes(s, s->streams[g], false, g0, g1, s->ws_g[g].p);
        }
    }
    for (int g = 0; g < G; g++) {
        HIP_CHECK(hipEventRecord(s->events[g], s->streams[g]));
        HIP_CHECK(hipStreamWaitEvent(stream, s->events[g], 0));
    }
}

void sampler_set_trial_theory(cmbs *s, int like_index, double *dl_end, long long ld_field, long long ld_walker) {
    if (like_index < 0 || like_index >= (int)s->likes.size()) fail(CMBL_ERR_ARG, "no likelihood %d", like_index);
    auto &e = s->end_theory[like_index];
    e.dl = dl_end;
    e.ld_field = ld_field;
    e.ld_walker = ld_walker;
}

// likelihood terms of set 1 (T rows, end theory) or set 2 (T2 rows, walker theory)
static void eval_likes_drag(cmbs *s, int set, hipStream_t stream) {
    // the fused window pass when both likelihoods read one buffer of this set
    bool fuse = false;
    if (s->tpass) {
        const int p = s->tp_like[0], c = s->tp_like[1];
        if (set == 1) {
            const auto &a = s->end_theory[p], &b = s->end_theory[c];
            fuse = a.dl == b.dl && a.ld_field == b.ld_field && a.ld_walker == b.ld_walker;
            if (fuse) launch_tpass(s, stream, a.dl, a.ld_field, a.ld_walker, s->dc.like_nuis);
        } else {
            double *nb2[MAXLIKE] = {};
            for (size_t i = 0; i < s->likes.size(); i++) nb2[i] = s->nuis_bufs2[i].as<double>();
            const LikeSlot &P = s->likes[p];
            fuse = true;
            launch_tpass(s, stream, P.dl, P.ld_field, P.ld_walker, nb2);
        }
    }
    for (size_t i = 0; i < s->likes.size(); i++) {
        auto &l = s->likes[i];
        const int nn = l.like->like->n_nuis;
        const double *dl = l.dl;
        long long ldf = l.ld_field, ldw = l.ld_walker;
        double *nb = s->dc.like_nuis[i];
        double *out = s->like_terms.as<double>() + i * (size_t)s->dc.ld;
        if (set == 1) {
            dl = s->end_theory[i].dl;
            ldf = s->end_theory[i].ld_field;
            ldw = s->end_theory[i].ld_walker;
        } else {
            nb = s->nuis_bufs2[i].as<double>();
            out = s->like_terms2.as<double>() + i * (size_t)s->dc.ld;
        }
        if (fuse && fused(s, i)) {
            l.like->like->after_window(s->W, nb, nn, out, s->like_ws[i].p, stream, false);
            continue;
        }
        l.like->like->loglike_batch(s->W, dl, ldf, ldw, nb, nn, out, s->ws.p, stream);
    }
}

// drag_staged_kernel's LDS image (0 when it would not fit a CU's 160 KB)
static size_t drag_lds_bytes(const cmbs *s) {
    const DevCfg &d = s->dc;
    const int nd_st = d.stage_R ? d.rows.ND : d.rows.ND - d.rows.RR;
    const int ni_st = d.stage_cyc ? d.rows.NI : d.rows.CYC;
    const int ntd = d.stage_cov ? d.tl.n_dbl : d.tl.covinv;
    const int nlk = (d.n_like + 1) & ~1, ndd = (drag_rows(d) + 1) & ~1;
    const size_t b = (size_t)(nd_st + ndd + 2 * nlk) * MB * 8 + (size_t)((ntd + 31) & ~31) * 8 +
                     (size_t)(ni_st + 4 + d.all_n) * MB * 4 + (size_t)((d.tl.n_int + 63) & ~63) * 4;
    return b <= 160 * 1024 ? b : 0;
}

template <int STAGE>
static void launch_drag(cmbs *s, const DragCfg &g, const HistRow &row, hipStream_t stream) {
    const size_t lds = drag_lds_bytes(s);
    timed_launch("drag_kernel", stream, [&](hipEvent_t e0, hipEvent_t e1) {
        if (lds && !s->drag_hbm)
            hipExtLaunchKernelGGL(drag_staged_kernel<STAGE>, dim3((s->W + MB - 1) / MB), dim3(MH_THREADS), lds, stream,
                                  e0, e1, 0, s->dc, g, row.p, row.t);
        else
            hipExtLaunchKernelGGL(drag_kernel<STAGE>, dim3((s->W + 63) / 64), dim3(64), 0, stream, e0, e1, 0, s->dc,
                                  g, row.p, row.t);
    });
    HIP_CHECK(hipGetLastError());
}

// Both evaluation sets of a drag's interpolation step (the end points T with
// the end theories, the start points T2 with the walkers' theories) as two
// launches instead of eight: the fused window pass over both theory sets
// (theory_window_pair, which also zeroes the tickets), then plik_lite's two
// in-launch-combined quadratic forms with both lensing chi^2s riding along
// (launch_qf_pair).  Set 2 works in its own workspaces (like_ws2).  False when
// the sets cannot be fused (then eval_likes_drag runs each).
static bool eval_likes_drag_pair(cmbs *s, hipStream_t stream, bool both = true) {
    if (!s->tpass || s->no_drag_pair) return false;
    int kq = -1, kg = -1;
    for (int k = 0; k < 2; k++) (s->tp_stage[k].kind == 1 ? kq : kg) = k;
    if (kq < 0 || kg < 0) return false;
    const int qi = s->tp_like[kq], gi = s->tp_like[kg];
    const auto &ea = s->end_theory[qi], &eb = s->end_theory[gi];
    if (ea.dl != eb.dl || ea.ld_field != eb.ld_field || ea.ld_walker != eb.ld_walker) return false;
    const LikeSlot &P = s->likes[qi];
    if (!s->tpass->vec_ok(ea.dl, ea.ld_field, ea.ld_walker) || !s->tpass->vec_ok(P.dl, P.ld_field, P.ld_walker))
        return false;
    const int W = s->W;
    for (int k = 0; k < 2; k++) {
        const int i = s->tp_like[k];
        const size_t need = s->likes[i].like->like->workspace_size(W);
        if (s->like_ws2[i].bytes < need) s->like_ws2[i].alloc(need);
    }
    Like &Q = *s->likes[qi].like->like;
    Like &G = *s->likes[gi].like->like;
    QFSource qa, qb;
    if (!Q.qf_source(qa, W, s->like_ws[qi].p) || !Q.qf_source(qb, W, s->like_ws2[qi].p)) return false;
    SmallGaussLaunch ga{}, gb{};
    const size_t ld = s->dc.ld;
    double *t1 = s->like_terms.as<double>(), *t2 = s->like_terms2.as<double>();
    if (!G.corun_small(ga, W, s->dc.like_nuis[gi], G.n_nuis, t1 + (size_t)gi * ld, s->like_ws[gi].p) ||
        !G.corun_small(gb, W, s->nuis_bufs2[gi].as<double>(), G.n_nuis, t2 + (size_t)gi * ld, s->like_ws2[gi].p))
        return false;
    TPOut oa[2], ob[2];
    for (int k = 0; k < 2; k++) {
        const int i = s->tp_like[k];
        const WinStage &st = s->tp_stage[k];
        Like &L = *s->likes[i].like->like;
        const long long ldn = std::max(1, L.n_nuis);
        oa[k] = TPOut{st.kind, st.cal_index, st.ld, 0, L.window_out(s->like_ws[i].p, W), st.X, s->dc.like_nuis[i], ldn};
        ob[k] = TPOut{st.kind, st.cal_index, st.ld, 0, L.window_out(s->like_ws2[i].p, W), st.X,
                      s->nuis_bufs2[i].as<double>(), ldn};
    }
    s->tpass->launch_pair(ea.dl, ea.ld_field, ea.ld_walker, oa, qa.counters, both ? P.dl : nullptr, P.ld_field,
                          P.ld_walker, ob, qb.counters, qa.n_counters, W, stream);
    launch_qf_pair(qa, t1 + (size_t)qi * ld, both ? &qb : nullptr, t2 + (size_t)qi * ld, W, &ga, both ? &gb : nullptr,
                   stream, "plik_quadform_pair");
    for (size_t i = 0; i < s->likes.size(); i++) {   // any other likelihood, one set after the other
        if (fused(s, i)) continue;
        auto &l = s->likes[i];
        const int nn = l.like->like->n_nuis;
        const auto &e = s->end_theory[i];
        l.like->like->loglike_batch(W, e.dl, e.ld_field, e.ld_walker, s->dc.like_nuis[i], nn, t1 + i * ld, s->ws.p,
                                    stream);
        if (both)
            l.like->like->loglike_batch(W, l.dl, l.ld_field, l.ld_walker, s->nuis_bufs2[i].as<double>(), nn,
                                        t2 + i * ld, s->ws.p, stream);
    }
    return true;
}

// Whether likelihood i's accepted-theory copy repeats an earlier likelihood's
// (the same end and walker theory buffers and strides: fused likelihoods
// usually read one): then it is skipped, the copy being idempotent
static bool same_theory_swap(const cmbs *s, int i) {
    const auto &e = s->end_theory[i];
    const auto &l = s->likes[i];
    for (int j = 0; j < i; j++) {
        const auto &ej = s->end_theory[j];
        const auto &lj = s->likes[j];
        if (ej.dl == e.dl && ej.ld_walker == e.ld_walker && lj.dl == l.dl && lj.ld_walker == l.ld_walker &&
            std::min(ej.ld_walker, lj.ld_walker) >= std::min(e.ld_walker, l.ld_walker))
            return true;
    }
    return false;
}

void sampler_step_drag(cmbs *s, int n_steps, double dragging_steps, cmbs_theory_fn fn, void *user,
                       hipStream_t stream) {
    rot_schedule_unknown(s);           // the drag proposals move the blocks' loop indices
    if (!s->started) fail(CMBL_ERR_ARG, "cmbs_set_start must be called before cmbs_step_drag");
    check_theory_fresh(s);
    if (n_steps <= 0) return;
    if (s->fast_n == 0 || s->slow_n == 0) {   // MCMC.f90:351-354: plain Metropolis
        sampler_step(s, n_steps, 0, stream);
        return;
    }
    const int nl = (int)s->likes.size();
    for (int i = 0; i < nl; i++)
        if (!s->end_theory[i].dl) fail(CMBL_ERR_ARG, "dragging needs an end-point theory buffer for likelihood %d", i);
    if (nl > 0 && !fn) fail(CMBL_ERR_ARG, "dragging with data likelihoods needs a theory function");
    const size_t ld = s->dc.ld;
    const int np = s->np;
    if (!s->drag_dd.p) {
        s->drag_dd.alloc((size_t)(3 * np + 4 + s->dc.max_blk + std::max<size_t>(1, s->likes.size())) * ld * 8);
        s->drag_di.alloc((size_t)(1 + s->all_n) * ld * 4);
        HIP_CHECK(hipMemset(s->drag_dd.p, 0, s->drag_dd.bytes));
        HIP_CHECK(hipMemset(s->drag_di.p, 0, s->drag_di.bytes));
        s->like_terms2.alloc(std::max<size_t>(1, s->likes.size()) * ld * 8);
        HIP_CHECK(hipMemset(s->like_terms2.p, 0, s->like_terms2.bytes));
        for (int i = 0; i < nl; i++)
            s->nuis_bufs2[i].alloc((size_t)std::max(s->likes[i].like->like->n_nuis, 1) * s->W * 8);
    }
    DragCfg g{};
    g.dd = s->drag_dd.as<double>();
    g.di = s->drag_di.as<int>();
    g.like_terms2 = s->like_terms2.as<double>();
    for (int i = 0; i < nl; i++) g.like_nuis2[i] = s->nuis_bufs2[i].as<double>();
    int interp = (int)std::lround(dragging_steps * s->fast_n) + 1;   // MCMC.f90:386
    if (interp < 2) interp = 2;
    g.interp = interp;
    if (const size_t lds = drag_lds_bytes(s))
        for (const void *k : {(const void *)drag_staged_kernel<0>, (const void *)drag_staged_kernel<1>,
                              (const void *)drag_staged_kernel<2>})
            HIP_CHECK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    for (int step = 0; step < n_steps; step++) {
        s->num_drag++;
        if (s->num_drag % s->dc.oversample_fast != 0) {   // FastParameterSample (:357-361)
            const bool m = s->mask_on;
            launch_mh(s, false, true, 1, HistRow{}, stream, 0, s->W, m);
            if (m) eval_likes_masked(s, stream);
            else eval_likes(s, stream, false, 0, s->W, s->ws.p);
            launch_mh(s, true, false, 1, next_hist(s), stream, 0, s->W, m);
            continue;
        }
        g.istep = 0;
        launch_drag<0>(s, g, HistRow{}, stream);
        if (nl > 0) {
            const double *Pend = s->dc.sd + (size_t)s->dc.rows.T * ld;
            if (fn(user, s->W, Pend, (long long)ld, stream) != 0) fail(CMBL_ERR_ARG, "theory function failed");
            if (!eval_likes_drag_pair(s, stream, false)) eval_likes_drag(s, 1, stream);
        }
        launch_drag<1>(s, g, HistRow{}, stream);
        for (int is = 1; is <= interp - 1; is++) {
            if (nl > 0 && !eval_likes_drag_pair(s, stream)) {
                eval_likes_drag(s, 1, stream);
                eval_likes_drag(s, 2, stream);
            }
            g.istep = is;
            const HistRow row = is == interp - 1 ? next_hist(s) : HistRow{};
            launch_drag<2>(s, g, row, stream);
        }
        s->theory_moved = s->theory_moved || nl > 0;
        for (int i = 0; i < nl; i++) {               // accepted drags keep the end theory
            const auto &e = s->end_theory[i];
            const auto &l = s->likes[i];
            const long long n = std::min(e.ld_walker, l.ld_walker) > 0 ? std::min(e.ld_walker, l.ld_walker)
                                                                        : 10 * l.ld_field;
            if (l.ld_walker == 0) fail(CMBL_ERR_ARG, "dragging needs per-walker theory rows (ld_walker > 0)");
            if (same_theory_swap(s, i)) continue;
            hipLaunchKernelGGL(drag_swap_theory, dim3(8, s->W), dim3(256), 0, stream, g.di, 4, s->W, e.dl,
                               e.ld_walker, const_cast<double *>(l.dl), l.ld_walker, n);
            HIP_CHECK(hipGetLastError());
        }
        // (every walker's dst is set again by the next drag's stage 0)
    }
}

// full TMetropolisSampler_GetNewSample steps (MCMC.f90:269-307) with the
// theory recomputed at every trial point: the caller's theory function fills
// the trial-theory buffers, the likelihoods run on them, and accepted walkers
// take the trial theory as their own
static void swap_accepted_theory(cmbs *s, hipStream_t stream) {
    const int *flag = s->dc.si + (size_t)s->dc.rows.ACCF * s->dc.ld;
    s->theory_moved = true;
    for (size_t i = 0; i < s->likes.size(); i++) {
        const auto &e = s->end_theory[i];
        const auto &l = s->likes[i];
        const long long n = std::min(e.ld_walker, l.ld_walker);
        if (same_theory_swap(s, (int)i)) continue;
        hipLaunchKernelGGL(drag_swap_theory, dim3(16, s->W), dim3(256), 0, stream, flag, 1, s->W, e.dl, e.ld_walker,
                           const_cast<double *>(l.dl), l.ld_walker, n);
        HIP_CHECK(hipGetLastError());
    }
}

void sampler_step_theory(cmbs *s, int n_steps, cmbs_theory_fn fn, void *user, hipStream_t stream) {
    if (!s->started) fail(CMBL_ERR_ARG, "cmbs_set_start must be called before cmbs_step_theory");
    check_theory_fresh(s);
    if (n_steps <= 0) return;
    if (s->likes.empty()) {
        sampler_step(s, n_steps, 0, stream);
        return;
    }
    if (!fn) fail(CMBL_ERR_ARG, "cmbs_step_theory needs a theory function");
    for (size_t i = 0; i < s->likes.size(); i++) {
        if (!s->end_theory[i].dl) fail(CMBL_ERR_ARG, "likelihood %zu has no trial-theory buffer", i);
        if (s->likes[i].ld_walker == 0) fail(CMBL_ERR_ARG, "slow steps need per-walker theory rows");
    }
    const double *Ptrial = s->dc.sd + (size_t)s->dc.rows.T * s->dc.ld;
    auto trial_likes = [&]() {
        if (fn(user, s->W, Ptrial, (long long)s->dc.ld, stream) != 0) fail(CMBL_ERR_ARG, "theory function failed");
        eval_likes_drag(s, 1, stream);
    };
    launch_mh(s, false, true, 0, HistRow{}, stream, 0, s->W);
    trial_likes();
    for (int k = 1; k < n_steps; k++) {
        launch_mh(s, true, true, 0, next_hist(s), stream, 0, s->W);
        swap_accepted_theory(s, stream);
        trial_likes();
    }
    launch_mh(s, true, false, 0, next_hist(s), stream, 0, s->W);
    swap_accepted_theory(s, stream);
}

// After a resume: the theory at every walker's current point (rows P) from the
// caller's theory function, copied into each likelihood's walker theory rows
// (the reference recomputes theory at the restart point too,
// GeneralSetup.f90:123-131).  The restored CurLike and per-likelihood terms are
// kept as saved, not re-evaluated: theory_fn must reproduce the theory the run
// had at those points (under a change mask, unchanged likelihoods keep their
// saved terms).
__global__ void copy_theory_rows(int W, const double *src, long long src_ld, double *dst, long long dst_ld, long long n)
{
    const int w = blockIdx.y;
    if (w >= W) return;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        dst[(long long)w * dst_ld + i] = src[(long long)w * src_ld + i];
}

void sampler_refresh_theory(cmbs *s, cmbs_theory_fn fn, void *user, hipStream_t stream) {
    if (!s->started) fail(CMBL_ERR_ARG, "no chain state: cmbs_set_start or cmbs_load_state first");
    if (!fn) fail(CMBL_ERR_ARG, "cmbs_refresh_theory needs a theory function");
    for (size_t i = 0; i < s->likes.size(); i++) {
        if (!s->end_theory[i].dl) fail(CMBL_ERR_ARG, "likelihood %zu has no trial-theory buffer", i);
        if (s->likes[i].ld_walker == 0) fail(CMBL_ERR_ARG, "per-walker theory rows needed (ld_walker > 0)");
    }
    const double *Pcur = s->dc.sd + (size_t)s->dc.rows.P * s->dc.ld;
    if (fn(user, s->W, Pcur, (long long)s->dc.ld, stream) != 0) fail(CMBL_ERR_ARG, "theory function failed");
    for (size_t i = 0; i < s->likes.size(); i++) {
        const auto &e = s->end_theory[i];
        const auto &l = s->likes[i];
        hipLaunchKernelGGL(copy_theory_rows, dim3(16, s->W), dim3(256), 0, stream, s->W, e.dl, e.ld_walker,
                           const_cast<double *>(l.dl), l.ld_walker, std::min(e.ld_walker, l.ld_walker));
        HIP_CHECK(hipGetLastError());
    }
    s->theory_stale = false;
}

void sampler_set_groups(cmbs *s, int n_groups) {
    {   // the groups step together: a common known loop index carries over to the new split
        const int v = s->rot_lp.empty() ? -1 : s->rot_lp[0];
        const bool same = std::all_of(s->rot_lp.begin(), s->rot_lp.end(), [v](int x) { return x == v; });
        std::fill(s->rot_lp.begin(), s->rot_lp.end(), same ? v : -1);
    }
    const int nblk = (s->W + NB - 1) / NB;
    if (n_groups < 1 || n_groups > MAXGROUPS) fail(CMBL_ERR_ARG, "n_groups must be in 1..%d", MAXGROUPS);
    if (n_groups > nblk) n_groups = nblk;
    s->grp0.assign(n_groups + 1, 0);
    for (int g = 0; g <= n_groups; g++) s->grp0[g] = std::min(s->W, (int)((long long)nblk * g / n_groups) * NB);
    for (int g = 0; g < n_groups; g++) {
        if (!s->streams[g]) HIP_CHECK(hipStreamCreateWithFlags(&s->streams[g], hipStreamNonBlocking));
        size_t ws = 0;
        for (auto &l : s->likes) ws = std::max(ws, l.like->like->workspace_size(s->grp0[g + 1] - s->grp0[g]));
        s->ws_g[g].alloc(ws);
    }
    for (auto &e : s->events)
        if (!e) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    s->n_groups = n_groups;
}

void sampler_enable_history(cmbs *s, int capacity) {
    s->hist.alloc((size_t)capacity * (s->n_used + 1) * s->W * 8);   // per step: P(params_used) rows, CurLike row
    s->hist_cap = capacity;
    s->hist_count = 0;
    if (!s->likes.empty()) {   // per step: each likelihood's -lnL at the current point
        s->hist_terms.alloc((size_t)capacity * s->likes.size() * s->W * 8);
        HIP_CHECK(hipMemset(s->hist_terms.p, 0, s->hist_terms.bytes));
    }
}

void sampler_history_stats(cmbs *s, int first, int last, double *means, double *covs, hipStream_t stream) {
    if (s->hist_cap == 0) fail(CMBL_ERR_ARG, "history not enabled");
    if (first < 0 || last < first || last >= s->hist_count || s->hist_count - first > s->hist_cap)
        fail(CMBL_ERR_ARG, "history rows [%d, %d] not available (count %d, capacity %d)", first, last,
             s->hist_count, s->hist_cap);
    const int n = s->n_used;
    const dim3 gm((s->W + 63) / 64), gc((s->W + 63) / 64, n), blk(64 * HS_PH);
    const double *h = s->hist.as<double>();
    auto run = [&](auto kmean, auto kcov) {
        hipLaunchKernelGGL(kmean, gm, blk, 0, stream, h, s->hist_cap, s->W, n, first, last, means);
        HIP_CHECK(hipGetLastError());
        hipLaunchKernelGGL(kcov, gc, blk, 0, stream, h, s->hist_cap, s->W, n, first, last, means, covs);
        HIP_CHECK(hipGetLastError());
    };
    if (n <= 8) run(hist_mean_kernel<8>, hist_cov_kernel<8>);
    else if (n <= 16) run(hist_mean_kernel<16>, hist_cov_kernel<16>);
    else if (n <= 32) run(hist_mean_kernel<32>, hist_cov_kernel<32>);
    else run(hist_mean_kernel<64>, hist_cov_kernel<64>);
}

void sampler_chain_moments(cmbs *s, int first, int last, const double *gmean, double *out, hipStream_t stream) {
    const int n = s->n_used;
    s->mom.grow((size_t)s->W * (n + n * n) * 8);
    double *means = s->mom.as<double>(), *covs = means + (size_t)s->W * n;
    sampler_history_stats(s, first, last, means, covs, stream);
    chain_moments_launch(means, covs, s->W, n, (double)(last - first + 1), nullptr, gmean, out, stream);
}

void sampler_history_host(cmbs *s, int first, int count, double *out) {
    if (s->hist_cap == 0) fail(CMBL_ERR_ARG, "history not enabled");
    const int oldest = std::max(0, s->hist_count - s->hist_cap);
    if (first < oldest || first + count > s->hist_count)
        fail(CMBL_ERR_ARG, "history rows [%d, %d) not kept (rows %d..%d)", first, first + count, oldest, s->hist_count - 1);
    HIP_CHECK(hipDeviceSynchronize());
    const size_t blk = (size_t)(s->n_used + 1) * s->W;
    for (int k = 0; k < count; k++) {
        const int slot = (first + k) % s->hist_cap;
        HIP_CHECK(hipMemcpy(out + (size_t)k * blk, s->hist.as<double>() + (size_t)slot * blk, blk * 8,
                            hipMemcpyDeviceToHost));
    }
}

void sampler_history_terms_host(cmbs *s, int first, int count, double *out) {
    if (s->hist_cap == 0) fail(CMBL_ERR_ARG, "history not enabled");
    const int oldest = std::max(0, s->hist_count - s->hist_cap);
    if (first < oldest || first + count > s->hist_count)
        fail(CMBL_ERR_ARG, "history rows [%d, %d) not kept (rows %d..%d)", first, first + count, oldest, s->hist_count - 1);
    const size_t blk = s->likes.size() * (size_t)s->W;
    if (blk == 0) return;
    HIP_CHECK(hipDeviceSynchronize());
    for (int k = 0; k < count; k++) {
        const int slot = (first + k) % s->hist_cap;
        HIP_CHECK(hipMemcpy(out + (size_t)k * blk, s->hist_terms.as<double>() + (size_t)slot * blk, blk * 8,
                            hipMemcpyDeviceToHost));
    }
}

// checkpoint resume of the history ring: rows [first, first + count) as
// written by sampler_history_host go back to their ring slots, and the ring
// continues at first + count (the samples the convergence test windows over,
// TMpiChainCollector_ReadState's Samples%LoadState, SampleCollector.f90:167)
void sampler_history_restore(cmbs *s, int first, int count, const double *in, const double *terms) {
    if (s->hist_cap == 0) fail(CMBL_ERR_ARG, "history not enabled");
    if (first < 0 || count < 0 || count > s->hist_cap)
        fail(CMBL_ERR_ARG, "history rows [%d, %d) do not fit the ring (capacity %d)", first, first + count,
             s->hist_cap);
    HIP_CHECK(hipDeviceSynchronize());
    const size_t blk = (size_t)(s->n_used + 1) * s->W;
    for (int k = 0; k < count; k++) {
        const int slot = (first + k) % s->hist_cap;
        HIP_CHECK(hipMemcpy(s->hist.as<double>() + (size_t)slot * blk, in + (size_t)k * blk, blk * 8,
                            hipMemcpyHostToDevice));
    }
    const size_t tblk = s->likes.size() * (size_t)s->W;
    if (terms && tblk)
        for (int k = 0; k < count; k++) {
            const int slot = (first + k) % s->hist_cap;
            HIP_CHECK(hipMemcpy(s->hist_terms.as<double>() + (size_t)slot * tblk, terms + (size_t)k * tblk,
                                tblk * 8, hipMemcpyHostToDevice));
        }
    s->hist_count = first + count;
}

void sampler_get_state_host(cmbs *s, double *P, double *cur_like, double *mult, int *num_accept) {
    HIP_CHECK(hipDeviceSynchronize());
    const int W = s->W, np = s->np;
    const size_t ld = s->dc.ld;
    const Rows &R = s->dc.rows;
    if (P) {
        std::vector<double> t((size_t)np * ld);
        HIP_CHECK(hipMemcpy(t.data(), s->dc.sd + (size_t)R.P * ld, t.size() * 8, hipMemcpyDeviceToHost));
        for (int w = 0; w < W; w++)
            for (int i = 0; i < np; i++) P[(size_t)w * np + i] = t[(size_t)i * ld + w];
    }
    if (cur_like) HIP_CHECK(hipMemcpy(cur_like, s->dc.sd + (size_t)R.L * ld, (size_t)W * 8, hipMemcpyDeviceToHost));
    if (mult) HIP_CHECK(hipMemcpy(mult, s->dc.sd + (size_t)R.M * ld, (size_t)W * 8, hipMemcpyDeviceToHost));
    if (num_accept)
        HIP_CHECK(hipMemcpy(num_accept, s->dc.si + (size_t)R.NACC * ld, (size_t)W * 4, hipMemcpyDeviceToHost));
}

// Checkpoint image of every walker's chain state: the reference's .chk holds
// num_sample / MaxLike / num_accept (MCMC.f90:98-114, 199-218) and the
// proposal matrix (propose.f90:308-325) and restarts from the last chain row
// with a fresh RNG (GeneralSetup.f90:123-131); this image holds the complete
// device state instead -- point, CurLike, multiplicity, accept count, RANMAR
// table and Gaussian1 cache, cyclic-index and rotation state, each
// likelihood's term at the point -- so a resumed run continues each chain
// exactly.  Layout: StateHeader, double rows [ND][W], int rows [NI][W],
// current terms [n_like][W].  The proposal covariance is the caller's part
// (cmbs_set_covariance before cmbs_load_state).
struct StateHeader {
    unsigned magic, version;
    int W, np, n_used, nblocks, all_n, slow_n, fast_n, R_total, ND, NI, n_like, theory_moved;
    int coll_cap, pad;      // sample-collector ring (0: not enabled) appended after the terms
    long long num_drag;
};
static constexpr unsigned STATE_MAGIC = 0x53424d43u;   // "CMBS"

size_t sampler_state_bytes(const cmbs *s) {
    const Rows &R = s->dc.rows;
    return sizeof(StateHeader) + (size_t)(R.ND + s->likes.size()) * s->W * 8 + (size_t)R.NI * s->W * 4 +
           sampler_collector_bytes(s);
}

static StateHeader state_header(const cmbs *s) {
    const Rows &R = s->dc.rows;
    return StateHeader{STATE_MAGIC, 2u, s->W, s->np, s->n_used, s->nblocks, s->all_n, s->slow_n, s->fast_n,
                       s->R_total, R.ND, R.NI, (int)s->likes.size(), s->theory_moved ? 1 : 0,
                       s->coll.enabled ? s->coll.cap : 0, 0, s->num_drag};
}

void sampler_save_state(cmbs *s, void *buf, size_t bytes) {
    if (!s->started) fail(CMBL_ERR_ARG, "no chain state yet: cmbs_set_start first");
    if (bytes < sampler_state_bytes(s)) fail(CMBL_ERR_ARG, "state buffer too small (%zu < %zu bytes)", bytes,
                                            sampler_state_bytes(s));
    HIP_CHECK(hipDeviceSynchronize());
    const Rows &R = s->dc.rows;
    const size_t ld = s->dc.ld, W = s->W;
    char *p = static_cast<char *>(buf);
    const StateHeader h = state_header(s);
    std::memcpy(p, &h, sizeof h);
    p += sizeof h;
    HIP_CHECK(hipMemcpy2D(p, W * 8, s->dc.sd, ld * 8, W * 8, R.ND, hipMemcpyDeviceToHost));
    p += (size_t)R.ND * W * 8;
    HIP_CHECK(hipMemcpy2D(p, W * 4, s->dc.si, ld * 4, W * 4, R.NI, hipMemcpyDeviceToHost));
    p += (size_t)R.NI * W * 4;
    if (!s->likes.empty())
        HIP_CHECK(hipMemcpy2D(p, W * 8, s->dc.cur_terms, ld * 8, W * 8, s->likes.size(), hipMemcpyDeviceToHost));
    p += s->likes.size() * W * 8;
    if (s->coll.enabled) sampler_collector_save(s, p);
}

void sampler_load_state(cmbs *s, const void *buf, size_t bytes) {
    rot_schedule_unknown(s);
    if (bytes < sizeof(StateHeader)) fail(CMBL_ERR_ARG, "state image too short");
    StateHeader h;
    std::memcpy(&h, buf, sizeof h);
    if (h.magic != STATE_MAGIC || h.version != 2u) fail(CMBL_ERR_FORMAT, "not a cmbs state image");
    const StateHeader m = state_header(s);
    if (h.W != m.W || h.np != m.np || h.n_used != m.n_used || h.nblocks != m.nblocks || h.all_n != m.all_n ||
        h.slow_n != m.slow_n || h.fast_n != m.fast_n || h.R_total != m.R_total || h.ND != m.ND || h.NI != m.NI ||
        h.n_like != m.n_like || h.coll_cap != m.coll_cap)
        fail(CMBL_ERR_ARG,
             "state image is for a different sampler (W %d np %d blocks %d likelihoods %d; this one W %d np %d "
             "blocks %d likelihoods %d)", h.W, h.np, h.nblocks, h.n_like, m.W, m.np, m.nblocks, m.n_like);
    if (bytes < sampler_state_bytes(s)) fail(CMBL_ERR_FORMAT, "state image truncated");
    const Rows &R = s->dc.rows;
    const size_t ld = s->dc.ld, W = s->W;
    const char *p = static_cast<const char *>(buf) + sizeof h;
    HIP_CHECK(hipDeviceSynchronize());
    HIP_CHECK(hipMemcpy2D(s->dc.sd, ld * 8, p, W * 8, W * 8, R.ND, hipMemcpyHostToDevice));
    p += (size_t)R.ND * W * 8;
    HIP_CHECK(hipMemcpy2D(s->dc.si, ld * 4, p, W * 4, W * 4, R.NI, hipMemcpyHostToDevice));
    p += (size_t)R.NI * W * 4;
    if (!s->likes.empty())
        HIP_CHECK(hipMemcpy2D(s->dc.cur_terms, ld * 8, p, W * 8, W * 8, s->likes.size(), hipMemcpyHostToDevice));
    p += s->likes.size() * W * 8;
    if (s->coll.enabled) sampler_collector_load(s, p);
    s->num_drag = h.num_drag;
    s->theory_moved = h.theory_moved != 0;
    s->theory_stale = s->theory_moved && !s->likes.empty();
    s->started = true;
}

}  // namespace cmamd

#ifdef CMAMD_STAMPS
extern "C" int cmamd_debug_uni_stamps(unsigned long long *host) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(cmamd::g_uni_stamps), sizeof(cmamd::g_uni_stamps)) == hipSuccess ? 0
                                                                                                               : -5;
}
extern "C" int cmamd_debug_stamps(unsigned long long *host) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(cmamd::g_stamps), sizeof(cmamd::g_stamps)) == hipSuccess ? 0 : -5;
}
#endif

// number of work items of the sampler's fused window pass (0: none); for tests
// (without one: minus the last set-up check passed)
extern "C" int cmamd_debug_rot_serial(cmbs *s, int mode) {   // 1: rotations by the serial path; 2: parallel, no speculative lanes
    if (!s) return -1;
    s->dc.rot_serial = mode;
    return 0;
}
extern "C" int cmamd_debug_stage_R(cmbs *s, int on) {     // rotation rows staged in mh_kernel's LDS image
    if (!s) return -1;
    s->stage_R_force = on;   // -1: set_mh_lds decides
    cmamd::set_mh_lds(s);
    return 0;
}
extern "C" int cmamd_debug_tp_items(const cmbs *s, int *out, int cap) {   // (field, l0, l1, steps, columns, blocks) per item
    if (!s || !s->tpass) return -1;
    const int n = std::min(cap, s->tpass->n_items());
    for (int k = 0; k < n; k++) {
        const cmamd::TPItem &it = s->tpass->item(k);
        const int v[6] = {it.field, it.l0, it.l1, it.nst, it.ncol, it.nsb};
        for (int q = 0; q < 6; q++) out[6 * k + q] = v[q];
    }
    return s->tpass->n_items();
}
extern "C" int cmamd_debug_pipeline(cmbs *s, int mode) {   // fast-step schedule (sampler_step): 0 unpipelined,
    if (!s || (mode != 0 && mode != 3)) return -1;   // 3 the unified launch (default), 0 unpipelined
    s->pipe_mode = mode;
    return 0;
}
extern "C" int cmamd_debug_lean(cmbs *s, int on) {   // the lean chain where it applies (1, default) or mh_body (0)
    if (!s) return CMBL_ERR_ARG;
    s->lean_off = !on;
    return 0;
}
extern "C" int cmamd_debug_corun(cmbs *s, int on) {     // the lensing chi^2 inside plik's quadratic-form launch
    if (!s) return -1;
    s->no_corun = !on;
    return 0;
}
extern "C" int cmamd_debug_tail_nosignal(cmbs *s, int on) {   // in-launch producers never arrive / publish (modes 1, 3)
    if (!s) return -1;
    s->tail_nosignal = on;
    return 0;
}
extern "C" int cmamd_debug_drag_pair(cmbs *s, int on) {   // both drag evaluation sets in two launches
    if (!s) return -1;
    s->no_drag_pair = on == 0;
    return 0;
}
extern "C" int cmamd_debug_drag_hbm(cmbs *s, int on) {   // the drag stages on the HBM state (no LDS image)
    if (!s) return -1;
    s->drag_hbm = on != 0;
    return 0;
}
extern "C" int cmamd_debug_pipe_status(cmbs *s) {   // the give-up word (synchronises the device)
    if (!s || !s->pipe_status_host) return -1;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    return *reinterpret_cast<volatile int *>(s->pipe_status_host);
}
extern "C" int cmamd_debug_tail(const cmbs *s) { return s ? s->tail_ready : 0; }   // W of the step tails' set-up
extern "C" int cmamd_debug_fused(const cmbs *s) { return !s ? 0 : s->tpass ? s->tpass->n_items() : -s->tp_why; }
