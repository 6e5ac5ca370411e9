// Batched Metropolis sampler: W independent CosmoMC chains, one per walker
// (one GPU thread per walker for the sequential per-chain logic), with the
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
// Walker state lives in HBM as structure-of-arrays ([field][walker]) so the
// per-thread state accesses of a wavefront fall on consecutive addresses.
#include <cmath>
#include <cstring>

#include "sampler.h"

namespace cmamd {

static constexpr double LOGZERO = CMBL_LOGZERO;
static constexpr int MAXP = 64;        // max parameters per chain handled in registers/stack
static constexpr int MAXBLK = 32;      // max block size

// ------------------------------------------------------------ RNG (RandUtils.f90)

struct Rng {
    double *u;      // column w of [97][W]
    int W;
    double c;
    int i97, j97, iset;
    double gset;
};

__device__ inline double U(const Rng &r, int i) { return r.u[(size_t)(i - 1) * r.W]; }

__device__ double ranmar(Rng &r)
{   // RandUtils.f90:350-374
    double uni = U(r, r.i97) - U(r, r.j97);
    if (uni < 0.0) uni += 1.0;
    r.u[(size_t)(r.i97 - 1) * r.W] = uni;
    if (--r.i97 == 0) r.i97 = 97;
    if (--r.j97 == 0) r.j97 = 97;
    const double cd = 7654321.0 / 16777216.0, cm = 16777213.0 / 16777216.0;
    r.c -= cd;
    if (r.c < 0.0) r.c += cm;
    uni -= r.c;
    if (uni < 0.0) uni += 1.0;
    return uni;
}

__device__ double gaussian1(Rng &r)
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

__device__ float randexp1(Rng &r)
{   // RandUtils.f90:189-233, REAL(4) arithmetic (no contraction: see -ffp-contract=off)
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

__device__ Rng load_rng(const DevCfg &c, int w)
{
    Rng r;
    r.u = c.rng_u + w;
    r.W = c.W;
    r.c = c.rng_c[w];
    r.i97 = c.rng_i97[w];
    r.j97 = c.rng_j97[w];
    r.iset = c.rng_iset[w];
    r.gset = c.rng_gset[w];
    return r;
}

__device__ void store_rng(const DevCfg &c, int w, const Rng &r)
{
    c.rng_c[w] = r.c;
    c.rng_i97[w] = r.i97;
    c.rng_j97[w] = r.j97;
    c.rng_iset[w] = r.iset;
    c.rng_gset[w] = r.gset;
}

__global__ void rng_init_kernel(DevCfg c, const int *ij, const int *kl)
{   // RMARIN, RandUtils.f90:286-348
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= c.W) return;
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
        c.rng_u[(size_t)ii * c.W + w] = s;
    }
    c.rng_c[w] = 362436.0 / 16777216.0;
    c.rng_i97[w] = 97;
    c.rng_j97[w] = 33;
    c.rng_iset[w] = 0;
    c.rng_gset[w] = 0.0;
}

// ------------------------------------------------------------ proposer (propose.f90)

// Per-walker arrays that need dynamic indexing live in LDS, one column per lane.
template <class T> struct Col {
    T *p;
    int s;   // stride between consecutive elements (the block size)
    __device__ T &operator[](int i) const { return p[i * s]; }
};

__device__ int cyc_next(const DevCfg &c, Rng &r, int w, int which, int n, int base, Col<int> tmp)
{   // CyclicIndexRandomizer%Next, propose.f90:75-86 (RandIndices RandUtils.f90:93-108)
    int *loopix = c.cyc_loopix + (size_t)which * c.W + w;
    const int lp = *loopix % n + 1;
    *loopix = lp;
    int *idx = c.cyc + (size_t)base * c.W + w;    // idx[k*W]
    if (lp == 1) {
        if (n == 1) {
            (void)ranmar(r);                        // ix = int(ranmar()*1)+1 = 1
            idx[0] = 1;
        } else {
            for (int i = 0; i < n; i++) tmp[i] = i + 1;
            for (int i = 1; i <= n; i++) {
                const int ix = (int)(ranmar(r) * (n + 1 - i)) + 1;
                idx[(size_t)(i - 1) * c.W] = tmp[ix - 1];
                tmp[ix - 1] = tmp[n + 1 - i - 1];
            }
        }
    }
    return idx[(size_t)(lp - 1) * c.W];
}

__device__ void rot_matrix(const DevCfg &c, Rng &r, double *R, int n, Col<double> vec)
{   // RotMatrix propose.f90:88-102 -> RandRotationD RandUtils.f90:133-153
    // R element (j,i) (row j) at R[(j*n+i)*W]
    const size_t W = c.W;
    if (n > 1) {
        for (int j = 0; j < n; j++) {
            double norm;
            for (;;) {
                for (int i = 0; i < n; i++) vec[i] = gaussian1(r);
                for (int i = 0; i < j; i++) {
                    double s = 0.0;
                    for (int k = 0; k < n; k++) s += vec[k] * R[(i * n + k) * W];
                    for (int k = 0; k < n; k++) vec[k] = vec[k] - s * R[(i * n + k) * W];
                }
                norm = 0.0;
                for (int k = 0; k < n; k++) norm += vec[k] * vec[k];
                if (norm > 1e-3) break;
            }
            const double sn = sqrt(norm);
            for (int k = 0; k < n; k++) R[(j * n + k) * W] = vec[k] / sn;
        }
    } else {
        for (int i = 0; i < n * n; i++) R[i * W] = 0.0;
        for (int i = 0; i < n; i++) R[(i * n + i) * W] = (ranmar(r) - 0.5) >= 0.0 ? 1.0 : -1.0;
    }
}

struct Scratch {
    Col<double> trial, vec;
    Col<int> itmp;
};

__device__ void block_proposal(const DevCfg &c, Rng &r, int w, int bi /*1-based*/, const Scratch &sc)
{   // GetBlockProposal :247-254 -> ProposeVec :105-120 -> Propose_r :122-139 -> UpdateParams :142-149
    const int b = bi - 1;
    const int n = c.blk_n[b];
    const size_t W = c.W;
    double *R = c.R + (size_t)c.blk_R_off[b] * W + w;
    int *loopix = c.blk_loopix + (size_t)b * W + w;
    int lp = *loopix;
    if (lp % n == 0) {
        rot_matrix(c, r, R, n, sc.vec);
        lp = 0;
    }
    lp++;
    *loopix = lp;
    double rf;
    if (ranmar(r) < 0.33) {
        rf = (double)randexp1(r);
    } else {
        const int m = n < 2 ? n : 2;
        rf = 0.0;
        for (int i = 0; i < m; i++) {
            const double g = gaussian1(r);
            rf += g * g;
        }
        rf = sqrt(rf / m);
    }
    const double scale = rf * c.propose_scale;
    // vec(k) = R(k, loopix) * (r * wid);  P(changed) += mapping_matrix . vec
    const int nc = c.blk_nchanged[b];
    const double *M = c.mapping + c.blk_map_off[b];
    const int *chg = c.changed + c.blk_changed_off[b];
    for (int j = 0; j < nc; j++) {
        double s = 0.0;
        for (int k = 0; k < n; k++) s += M[j * n + k] * (R[((size_t)k * n + (lp - 1)) * W] * scale);
        sc.trial[chg[j]] += s;
    }
}

__device__ void proposal_fast(const DevCfg &c, Rng &r, int w, const Scratch &sc)
{   // :283-289
    const int k = cyc_next(c, r, w, 2, c.fast_n, c.all_n + c.slow_n, sc.itmp);
    block_proposal(c, r, w, c.proposer_for_index[c.slow_n + k - 1], sc);
}

__device__ void proposal_slow(const DevCfg &c, Rng &r, int w, const Scratch &sc)
{   // :275-281
    const int k = cyc_next(c, r, w, 1, c.slow_n, c.all_n, sc.itmp);
    block_proposal(c, r, w, c.proposer_for_index[k - 1], sc);
}

__device__ void proposal(const DevCfg &c, Rng &r, int w, const Scratch &sc)
{   // GetProposal :257-273
    int fix = c.fast_ix[w];
    if (fix != 0) {
        proposal_fast(c, r, w, sc);
        fix--;
    } else if (cyc_next(c, r, w, 0, c.all_n, 0, sc.itmp) > c.slow_n) {
        proposal_fast(c, r, w, sc);
        fix = c.oversample_fast - 1;
    } else {
        proposal_slow(c, r, w, sc);
    }
    c.fast_ix[w] = fix;
}

// ------------------------------------------------------------ likelihood assembly

template <class Q> __device__ double target_like(const DevCfg &c, int w, const Q &q)
{   // GetLogLike calclike.f90:136-151 with AddLikeTemp :82-94
    for (int i = 0; i < c.np; i++)
        if (q[i] > c.pmax[i] || q[i] < c.pmin[i]) return LOGZERO;   // GetLogLikeBounds :97-109
    double main = 0.0;
    if (c.test_like) {                                               // TestLikelihoodFunction :180-199
        const int n = c.n_used;
        double d = 0.0;
        for (int i = 0; i < n; i++) {
            double s = 0.0;
            for (int j = 0; j < n; j++)
                s += c.test_covinv[i * n + j] * (q[c.params_used[j]] - c.center[c.params_used[j]]);
            d += (q[c.params_used[i]] - c.center[c.params_used[i]]) * s;
        }
        main = d / 2.0;
    }
    for (int l = 0; l < c.n_like; l++) {                             // LogLikeWithTheorySet :374-387
        const double v = c.like_terms[(size_t)l * c.W + w];
        if (v == LOGZERO) return LOGZERO;
        main += v;
    }
    double like = main / c.temperature;
    if (c.has_priors) {                                              // GetLogPriors :111-134
        double pri = 0.0;
        for (int i = 0; i < c.np; i++)
            if (c.prior_std[i] != 0.0) {
                const double z = (q[i] - c.prior_mean[i]) / c.prior_std[i];
                pri += z * z;
            }
        like = like + (pri / 2.0) / c.temperature;
    }
    return like;
}

// One launch per Metropolis step boundary: accept/reject the pending trial
// (MetropolisAccept MCMC.f90:119-131 + MoveDone :166-190), then propose the
// next trial (GetProposal / GetProposalFast) and scatter its nuisance
// parameters for the likelihood kernels.  One 64-lane wavefront per 64
// walkers; the walker's RANMAR state (97 doubles) is staged in LDS with one
// coalesced pass in and out, so the sequential RNG calls never wait on HBM.
template <bool ACCEPT, bool PROPOSE>
__global__ __launch_bounds__(64) void mh_kernel(DevCfg c, int fast_only, double *hist_row)
{
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int lane = threadIdx.x;
    const int w = blockIdx.x * 64 + lane;
    const bool act = w < c.W;
    const int wc = act ? w : c.W - 1;
    double *ul = lds;                           // [97][64]
    double *tl = lds + 97 * 64;                 // [np][64]
    double *vl = tl + c.np * 64;                // [max_blk][64]
    int *il = reinterpret_cast<int *>(vl + c.max_blk * 64);   // [all_n][64]
    for (int i = 0; i < 97; i++) ul[i * 64 + lane] = c.rng_u[(size_t)i * c.W + wc];
    for (int i = 0; i < c.np; i++) tl[i * 64 + lane] = c.trial[(size_t)i * c.W + wc];
    if (!act) return;
    Rng r;
    r.u = ul + lane;
    r.W = 64;
    r.c = c.rng_c[w];
    r.i97 = c.rng_i97[w];
    r.j97 = c.rng_j97[w];
    r.iset = c.rng_iset[w];
    r.gset = c.rng_gset[w];
    Scratch sc{Col<double>{tl + lane, 64}, Col<double>{vl + lane, 64}, Col<int>{il + lane, 64}};
    if (ACCEPT) {
        const double like = target_like(c, w, sc.trial);
        const double cur = c.cur_like[w];
        bool acc = false;
        if (like != LOGZERO) {
            acc = cur > like;
            if (!acc) acc = (double)randexp1(r) > like - cur;
        }
        if (acc) {
            if (c.mult[w] > 0) c.num_accept[w] += 1;
            c.mult[w] = 1.0;
            for (int i = 0; i < c.np; i++) c.P[(size_t)i * c.W + w] = sc.trial[i];
            c.cur_like[w] = like;
        } else {
            c.mult[w] += 1.0;
            for (int i = 0; i < c.np; i++) sc.trial[i] = c.P[(size_t)i * c.W + w];
        }
        if (hist_row)
            for (int i = 0; i < c.n_used; i++) hist_row[(size_t)i * c.W + w] = sc.trial[c.params_used[i]];
    } else if (PROPOSE) {
        for (int i = 0; i < c.np; i++) sc.trial[i] = c.P[(size_t)i * c.W + w];   // Trial = CurParams
    }
    if (PROPOSE) {
        if (fast_only) proposal_fast(c, r, w, sc);
        else proposal(c, r, w, sc);
        for (int i = 0; i < c.np; i++) c.trial[(size_t)i * c.W + w] = sc.trial[i];
        for (int l = 0; l < c.n_like; l++)
            for (int k = 0; k < c.like_nn[l]; k++)
                c.like_nuis[l][(size_t)w * c.like_nn[l] + k] = sc.trial[c.like_nuis0[l] + k];
    }
    c.rng_c[w] = r.c;
    c.rng_i97[w] = r.i97;
    c.rng_j97[w] = r.j97;
    c.rng_iset[w] = r.iset;
    c.rng_gset[w] = r.gset;
    for (int i = 0; i < 97; i++) c.rng_u[(size_t)i * c.W + w] = ul[i * 64 + lane];
}

__global__ void start_kernel(DevCfg c)
{
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= c.W) return;
    Col<double> q{c.trial + w, c.W};
    c.cur_like[w] = target_like(c, w, q);
    for (int i = 0; i < c.np; i++) c.P[(size_t)i * c.W + w] = q[i];
    c.mult[w] = 0.0;
    c.num_accept[w] = 0;
}

// scatter the nuisance slice of every walker's trial point: out[w][k] = trial[nuis0 + k][w]
__global__ void gather_nuis(const double *trial, int W, int nuis0, int n_nuis, double *out)
{
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= W) return;
    for (int k = 0; k < n_nuis; k++) out[(size_t)w * n_nuis + k] = trial[(size_t)(nuis0 + k) * W + w];
}

__global__ void hist_stats_kernel(const double *hist, int cap, int W, int n, int first, int last,
                                  double *means, double *covs)
{   // per-chain mean/cov over rows first..last (SampleCollector.f90:235-246)
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= W) return;
    const int cnt = last - first + 1;
    double m[MAXP];
    for (int i = 0; i < n; i++) m[i] = 0.0;
    for (int t = first; t <= last; t++) {
        const double *row = hist + (size_t)(t % cap) * n * W;
        for (int i = 0; i < n; i++) m[i] += row[(size_t)i * W + w];
    }
    for (int i = 0; i < n; i++) {
        m[i] /= cnt;
        means[(size_t)w * n + i] = m[i];
    }
    double *C = covs + (size_t)w * n * n;
    for (int i = 0; i < n * n; i++) C[i] = 0.0;
    for (int t = first; t <= last; t++) {
        const double *row = hist + (size_t)(t % cap) * n * W;
        double d[MAXP];
        for (int i = 0; i < n; i++) d[i] = row[(size_t)i * W + w] - m[i];
        for (int j = 0; j < n; j++)
            for (int i = 0; i < n; i++) C[i * n + j] += d[i] * d[j];
    }
    for (int i = 0; i < n * n; i++) C[i] /= cnt;
}


static size_t mh_lds_bytes(const cmbs *s) {
    return (size_t)(97 + s->np + s->dc.max_blk) * 64 * 8 + (size_t)s->all_n * 64 * 4;
}

static size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

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
    if (s->fast_n > MAXP || s->all_n > MAXP) fail(CMBL_ERR_ARG, "too many parameters");

    // ---- device tables
    const int np = s->np, W = s->W, nb = s->nblocks;
    std::vector<size_t> offs;
    size_t tot = 0;
    auto add = [&](size_t bytes) {
        offs.push_back(tot);
        tot += align_up(bytes);
    };
    add(nb * 4);                      // 0 blk_n
    add(nb * 4);                      // 1 blk_nchanged
    add(nb * 4);                      // 2 blk_changed_off
    add(nb * 4);                      // 3 blk_map_off
    add(nb * 4);                      // 4 blk_R_off
    add(s->changed.size() * 4);       // 5 changed
    add((size_t)s->map_total * 8);    // 6 mapping
    add(s->all_n * 4);                // 7 proposer_for_index
    add(np * 8);                      // 8 pmin
    add(np * 8);                      // 9 pmax
    add(np * 8);                      // 10 prior_mean
    add(np * 8);                      // 11 prior_std
    add(s->n_used * 4);               // 12 params_used (0-based)
    s->tables.alloc(tot);
    char *base = s->tables.as<char>();
    auto up = [&](int k, const void *src, size_t bytes) {
        if (bytes) HIP_CHECK(hipMemcpy(base + offs[k], src, bytes, hipMemcpyHostToDevice));
    };
    up(0, s->blk_n.data(), nb * 4);
    up(1, s->blk_nchanged.data(), nb * 4);
    up(2, s->blk_changed_off.data(), nb * 4);
    up(3, s->blk_map_off.data(), nb * 4);
    up(4, s->blk_R_off.data(), nb * 4);
    up(5, s->changed.data(), s->changed.size() * 4);
    up(7, s->proposer_for_index.data(), s->all_n * 4);
    up(8, cfg->pmin, np * 8);
    up(9, cfg->pmax, np * 8);
    std::vector<double> pm(np, 0.0), ps(np, 0.0);
    bool has_pri = false;
    if (cfg->prior_mean && cfg->prior_std) {
        for (int i = 0; i < np; i++) {
            pm[i] = cfg->prior_mean[i];
            ps[i] = cfg->prior_std[i];
            has_pri |= ps[i] != 0.0;
        }
    }
    up(10, pm.data(), np * 8);
    up(11, ps.data(), np * 8);
    std::vector<int> pu0(s->n_used);
    for (int i = 0; i < s->n_used; i++) pu0[i] = s->params_used[i] - 1;
    up(12, pu0.data(), s->n_used * 4);

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
    d.blk_n = (const int *)(base + offs[0]);
    d.blk_nchanged = (const int *)(base + offs[1]);
    d.blk_changed_off = (const int *)(base + offs[2]);
    d.blk_map_off = (const int *)(base + offs[3]);
    d.blk_R_off = (const int *)(base + offs[4]);
    d.changed = (const int *)(base + offs[5]);
    d.mapping = (const double *)(base + offs[6]);
    d.proposer_for_index = (const int *)(base + offs[7]);
    d.pmin = (const double *)(base + offs[8]);
    d.pmax = (const double *)(base + offs[9]);
    d.prior_mean = (const double *)(base + offs[10]);
    d.prior_std = (const double *)(base + offs[11]);
    d.params_used = (const int *)(base + offs[12]);
    d.has_priors = has_pri;
    d.R_total = s->R_total;
    d.max_blk = 1;
    for (int bn : s->blk_n) d.max_blk = std::max(d.max_blk, bn);
    {
        const int lds = (int)mh_lds_bytes(s);
        HIP_CHECK(hipFuncSetAttribute((const void *)mh_kernel<true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        HIP_CHECK(hipFuncSetAttribute((const void *)mh_kernel<true, false>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        HIP_CHECK(hipFuncSetAttribute((const void *)mh_kernel<false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    }

    // ---- per-walker state
    offs.clear();
    tot = 0;
    const int ncyc = s->all_n + s->slow_n + s->fast_n;
    add((size_t)97 * W * 8);          // 0 rng_u
    add((size_t)W * 8);               // 1 rng_c
    add((size_t)W * 8);               // 2 rng_gset
    add((size_t)W * 4);               // 3 i97
    add((size_t)W * 4);               // 4 j97
    add((size_t)W * 4);               // 5 iset
    add((size_t)s->R_total * W * 8);  // 6 R
    add((size_t)nb * W * 4);          // 7 blk_loopix
    add((size_t)ncyc * W * 4);        // 8 cyc
    add((size_t)3 * W * 4);           // 9 cyc_loopix
    add((size_t)W * 4);               // 10 fast_ix
    add((size_t)np * W * 8);          // 11 P
    add((size_t)np * W * 8);          // 12 trial
    add((size_t)W * 8);               // 13 cur_like
    add((size_t)W * 8);               // 14 mult
    add((size_t)W * 4);               // 15 num_accept
    s->state.alloc(tot);
    HIP_CHECK(hipMemset(s->state.p, 0, tot));
    base = s->state.as<char>();
    d.rng_u = (double *)(base + offs[0]);
    d.rng_c = (double *)(base + offs[1]);
    d.rng_gset = (double *)(base + offs[2]);
    d.rng_i97 = (int *)(base + offs[3]);
    d.rng_j97 = (int *)(base + offs[4]);
    d.rng_iset = (int *)(base + offs[5]);
    d.R = (double *)(base + offs[6]);
    d.blk_loopix = (int *)(base + offs[7]);
    d.cyc = (int *)(base + offs[8]);
    d.cyc_loopix = (int *)(base + offs[9]);
    d.fast_ix = (int *)(base + offs[10]);
    d.P = (double *)(base + offs[11]);
    d.trial = (double *)(base + offs[12]);
    d.cur_like = (double *)(base + offs[13]);
    d.mult = (double *)(base + offs[14]);
    d.num_accept = (int *)(base + offs[15]);

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
    std::vector<double> map(s->map_total);
    int uoff = 0;
    for (int i = 0; i < s->nblocks; i++) {
        const int bn = s->blk_n[i], st = s->blk_start[i], nc = s->blk_nchanged[i];
        for (int j = 0; j < nc; j++)
            for (int k = 0; k < bn; k++)
                map[s->blk_map_off[i] + j * bn + k] =
                    sig[s->used_params_changed_all[uoff + j] - 1] * L[(st - 1 + j) * na + (st - 1 + k)];
        uoff += nc;
    }
    HIP_CHECK(hipMemcpy(const_cast<double *>(s->dc.mapping), map.data(), map.size() * 8, hipMemcpyHostToDevice));
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
    s->covinv.alloc(T.size() * 8);
    s->covinv.upload(T.data(), T.size() * 8);
    s->center.alloc(s->np * 8);
    s->center.upload(center, s->np * 8);
    s->dc.test_like = 1;
    s->dc.test_covinv = s->covinv.as<double>();
    s->dc.center = s->center.as<double>();
}

void sampler_add_likelihood(cmbs *s, cmbl_t *like, int nuis_index0, const double *dl, long long ld_field,
                            long long ld_walker) {
    if (!like) fail(CMBL_ERR_ARG, "null likelihood");
    const int nn = like->like->n_nuis;
    if (nuis_index0 < 1 || nuis_index0 - 1 + nn > s->np) fail(CMBL_ERR_ARG, "nuisance indices out of range");
    if ((int)s->likes.size() >= MAXLIKE) fail(CMBL_ERR_ARG, "at most %d likelihoods per sampler", MAXLIKE);
    const int li = (int)s->likes.size();
    s->likes.push_back({like, nuis_index0 - 1, dl, ld_field, ld_walker});
    s->like_terms.alloc(s->likes.size() * (size_t)s->W * 8);
    s->dc.n_like = (int)s->likes.size();
    s->dc.like_terms = s->like_terms.as<double>();
    s->nuis_bufs[li].alloc((size_t)std::max(nn, 1) * s->W * 8);
    s->dc.like_nuis[li] = s->nuis_bufs[li].as<double>();
    s->dc.like_nuis0[li] = nuis_index0 - 1;
    s->dc.like_nn[li] = nn;
    size_t maxws = 0;
    for (auto &l : s->likes) maxws = std::max(maxws, l.like->like->workspace_size(s->W));
    s->ws.alloc(maxws);
}

static void eval_likes(cmbs *s, hipStream_t stream, bool gather) {
    for (size_t i = 0; i < s->likes.size(); i++) {
        auto &l = s->likes[i];
        const int nn = l.like->like->n_nuis;
        double *nb = s->dc.like_nuis[i];
        if (gather) {   // mh_kernel scatters the nuisance slices itself on every step
            hipLaunchKernelGGL(gather_nuis, dim3((s->W + 255) / 256), dim3(256), 0, stream, s->dc.trial, s->W,
                               l.nuis0, nn, nb);
            HIP_CHECK(hipGetLastError());
        }
        l.like->like->loglike_batch(s->W, l.dl, l.ld_field, l.ld_walker, nb, nn,
                                    s->like_terms.as<double>() + i * (size_t)s->W, s->ws.p, stream);
    }
}

static void launch_mh(cmbs *s, bool accept, bool propose, int fast_only, double *row, hipStream_t stream) {
    const dim3 g((s->W + 63) / 64), b(64);
    const size_t lds = mh_lds_bytes(s);
    timed_launch("mh_kernel", stream, [&] {
        if (accept && propose)
            hipLaunchKernelGGL((mh_kernel<true, true>), g, b, lds, stream, s->dc, fast_only, row);
        else if (accept)
            hipLaunchKernelGGL((mh_kernel<true, false>), g, b, lds, stream, s->dc, fast_only, row);
        else
            hipLaunchKernelGGL((mh_kernel<false, true>), g, b, lds, stream, s->dc, fast_only, row);
    });
    HIP_CHECK(hipGetLastError());
}

void sampler_set_start(cmbs *s, const double *P0, hipStream_t stream) {
    // host [W][np] -> device trial [np][W]
    std::vector<double> t((size_t)s->np * s->W);
    for (int w = 0; w < s->W; w++)
        for (int i = 0; i < s->np; i++) t[(size_t)i * s->W + w] = P0[(size_t)w * s->np + i];
    HIP_CHECK(hipMemcpyAsync(s->dc.trial, t.data(), t.size() * 8, hipMemcpyHostToDevice, stream));
    eval_likes(s, stream, true);
    hipLaunchKernelGGL(start_kernel, dim3((s->W + 255) / 256), dim3(256), 0, stream, s->dc);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipStreamSynchronize(stream));
    s->started = true;
}

void sampler_step(cmbs *s, int n_steps, int fast_only, hipStream_t stream) {
    if (!s->started) fail(CMBL_ERR_ARG, "cmbs_set_start must be called before cmbs_step");
    if (fast_only && s->fast_n == 0) fail(CMBL_ERR_ARG, "no fast parameters");
    if (n_steps <= 0) return;
    auto next_row = [&]() -> double * {
        if (s->hist_cap == 0) return nullptr;
        double *row = s->hist.as<double>() + (size_t)(s->hist_count % s->hist_cap) * s->n_used * s->W;
        s->hist_count++;
        return row;
    };
    // propose(1) | likes | accept(1)+propose(2) | likes | ... | likes | accept(n)
    launch_mh(s, false, true, fast_only, nullptr, stream);
    eval_likes(s, stream, false);
    for (int k = 1; k < n_steps; k++) {
        launch_mh(s, true, true, fast_only, next_row(), stream);
        eval_likes(s, stream, false);
    }
    launch_mh(s, true, false, fast_only, next_row(), stream);
}

void sampler_enable_history(cmbs *s, int capacity) {
    s->hist.alloc((size_t)capacity * s->n_used * s->W * 8);
    s->hist_cap = capacity;
    s->hist_count = 0;
}

void sampler_history_stats(cmbs *s, int first, int last, double *means, double *covs, hipStream_t stream) {
    if (s->hist_cap == 0) fail(CMBL_ERR_ARG, "history not enabled");
    if (first < 0 || last < first || last >= s->hist_count || s->hist_count - first > s->hist_cap)
        fail(CMBL_ERR_ARG, "history rows [%d, %d] not available (count %d, capacity %d)", first, last,
             s->hist_count, s->hist_cap);
    hipLaunchKernelGGL(hist_stats_kernel, dim3((s->W + 127) / 128), dim3(128), 0, stream, s->hist.as<double>(),
                       s->hist_cap, s->W, s->n_used, first, last, means, covs);
    HIP_CHECK(hipGetLastError());
}

}  // namespace cmamd
