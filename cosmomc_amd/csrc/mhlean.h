// The lean Metropolis chain: accept / propose for fast-only steps whose only
// fast parameter is a one-parameter block (BASELINE configs[2]'s calPlanck,
// the headline workload).  Included by sampler.hip after the RNG, the LDS-DMA
// helpers and the deferred-combine helpers.
//
// Per walker this is the same arithmetic, in the same order, as mh_body on
// the same state (MetropolisAccept MCMC.f90:119-131, MoveDone :166-190,
// GetLogLike calclike.f90:136-151, GetProposalFast propose.f90:283-289 with
// the one-parameter block's RotMatrix :88-102 and Propose_r :122-139,
// UpdateParams :142-149), so the chains are bit-identical; what differs is
// how the state moves:
//   * the block's rows, changed parameters, mapping column and the nuisance
//     indices come from the kernel arguments (DevCfg::lean), not from LDS
//     table lookups, and the chain is straight-line code for that block;
//   * only the RANMAR ring, P / trial / CurLike / mult and the RNG indices are
//     staged (LDS-DMA); the rotation rows, cyclic-index permutations and the
//     shared tables are not;
//   * nothing is written back wholesale: the chain lanes store the rows they
//     changed, and after one barrier the thread groups store the ring entries
//     the draws overwrote (counted per walker, Rng::nd), P and the trial rows
//     and the history row, 16 walkers per 128-byte store.
// The trial calibrations are published straight after the proposal.
// (included inside namespace cmamd)
#pragma once

template <bool ACCEPT, bool PROPOSE>
__device__ __forceinline__ void mh_lean(const DevCfg &c, double *hist_row, double *hist_terms, int blk0, double *lds,
                                        int bx, const TailWait *tw)
{
    const Rows &R = c.rows;
    const LeanCfg &L = c.lean;
    const int lane = threadIdx.x % MB, grp = threadIdx.x / MB;
    const int wl64 = threadIdx.x & 63, wave = threadIdx.x >> 6, nwave = MH_THREADS / 64;
    const int wb = (blk0 + bx) * MB;
    const int w = wb + lane;
    const bool act = w < c.W;
    const size_t W = c.ld;
    const int np = c.np;
    // LDS: sd rows [0, R.R) (ring, c, gset) and [P, ND) (P, trial, CurLike, mult) | si rows [0, 8) |
    // deferred group sums | squared prior z | bounds verdict | per-walker draw count and first ring index
    const int nd_lo = R.R, nd_hi = R.ND - R.P;
    double *sd = lds;                                             // [nd_lo + nd_hi][MB]
    double *sp = sd + (size_t)nd_lo * MB;                         // row P at 0, trial at np, CurLike 2np, mult 2np+1
    double *dq = sp + (size_t)nd_hi * MB;                         // [n_def][QF_GROUPS + 1][MB]
    double *zz = dq + (size_t)MAXDEF * (QF_GROUPS + 1) * MB;      // [np][MB]
    int *si = reinterpret_cast<int *>(zz + (size_t)np * MB);      // [8][MB]
    int *oobw = si + 8 * MB;                                      // [MB]
    int *ndw = oobw + MB;                                         // [MB] draws this step
    int *i0w = ndw + MB;                                          // [MB] i97 before them
    if (threadIdx.x < MB) oobw[threadIdx.x] = 0;
    if (PROPOSE && c.rot_defer && bx == 0 && threadIdx.x == 0)   // as mh_body: the other rotation list restarts
        c.rot_cnt[2 * (blk0 * MB / 64) + (c.rot_par ^ 1)] = 0;

    STAMP(0);
    dma_rows_f64(sd, 0, c.sd, 0, nd_lo, W, wb, wl64, wave, nwave);
    dma_rows_f64(sd, nd_lo, c.sd, R.P, nd_hi, W, wb, wl64, wave, nwave);
    dma_rows_i32(si, c.si, 8, W, wb, wl64, wave, nwave);
    // the thread groups' loads, in flight beside the image: each group's
    // parameters' bounds and prior (GetLogLikeBounds / GetLogPriors); after the
    // unified launch's wait (tw), its split-K group sum of every deferred likelihood
    constexpr int PG = MAXP / NV;                                 // parameters per group at most
    double lo[PG], hi[PG], mu[PG], sg[PG];
    const double *td = c.tab_d;
#pragma unroll
    for (int u = 0; u < PG; u++) {
        const int i = grp + u * NV;
        if (ACCEPT && i < np) {
            lo[u] = td[c.tl.pmin + i];
            hi[u] = td[c.tl.pmax + i];
            mu[u] = td[c.tl.pmean + i];
            sg[u] = td[c.tl.pstd + i];
        }
    }
    int pu[PG];                                                   // the history row's parameters
    if (ACCEPT && hist_row) {
#pragma unroll
        for (int u = 0; u < PG; u++) {
            const int i = grp + u * NV;
            if (i < c.n_used) pu[u] = c.tab_i[c.tl.params_used + i];
        }
    }
    if (tw) tail_wait(*tw, wb / 64);   // the trial's terms below come from this launch's producers
    if (ACCEPT && c.n_def) {
        const int tile = wb / QF_TILE, col = wb % QF_TILE + lane;
        for (int d = 0; d < MAXDEF; d++) {
            if (d >= c.n_def) break;
            const double *tp = c.def_part[d] + (size_t)tile * c.def_items[d] * QF_TILE;
            double *row = dq + (size_t)d * (QF_GROUPS + 1) * MB;
            if (grp < QF_GROUPS) row[(size_t)grp * MB + lane] = qf_group_sum(tp, c.def_items[d], grp, col);
            if (grp == NV - 1) row[(size_t)QF_GROUPS * MB + lane] = (c.def_add[d] && act) ? c.def_add[d][w] : 0.0;
        }
    }
    // the chain lanes' own loads: the trial's likelihood terms and, for the
    // history, the current point's
    double lk[MAXLIKE], ct[MAXLIKE];
    if (ACCEPT && grp == 0 && act) {
#pragma unroll
        for (int l = 0; l < MAXLIKE; l++)
            if (l < c.n_like) {
                lk[l] = c.like_terms[(size_t)l * W + w];
                if (hist_terms) ct[l] = c.cur_terms[(size_t)l * W + w];
            }
    }
    STAMP(1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const double *trial_l = sp + (size_t)np * MB + lane;         // trial row i at trial_l[i * MB]
    if (ACCEPT && act) {   // bounds and squared prior z of the trial, one group per parameter
        int oob = 0;
#pragma unroll
        for (int u = 0; u < PG; u++) {
            const int i = grp + u * NV;
            if (i < np) {
                const double qv = trial_l[(size_t)i * MB];
                if (qv > hi[u] || qv < lo[u]) oob = 1;
                double z2 = 0.0;
                if (c.has_priors && sg[u] != 0.0) {
                    const double z = (qv - mu[u]) / sg[u];
                    z2 = z * z;
                }
                zz[(size_t)i * MB + lane] = z2;
            }
        }
        if (oob) atomicOr(&oobw[lane], 1);
    }
    if (ACCEPT) __syncthreads();
    STAMP(2);

    if (grp == 0 && act) {
        Rng r;
        r.u = Col<double>{sd + (size_t)R.U * MB + lane, MB};
        r.c = sd[(size_t)R.C * MB + lane];
        r.gset = sd[(size_t)R.G * MB + lane];
        r.i97 = si[(size_t)R.I97 * MB + lane];
        r.j97 = si[(size_t)R.J97 * MB + lane];
        r.iset = si[(size_t)R.ISET * MB + lane];
        r.nd = 0;
        const int i97_0 = r.i97;
        double *P = sp + lane;                                    // row i at P[i * MB]
        double *T = sp + (size_t)np * MB + lane;
        double cur = sp[(size_t)(2 * np) * MB + lane];
        double mult = sp[(size_t)(2 * np + 1) * MB + lane];
        int nacc = si[(size_t)R.NACC * MB + lane];
        bool moved = false;
        if (ACCEPT) {
            for (int d = 0; d < MAXDEF; d++) {   // the deferred combines, in quadform.h's fixed order
                if (d >= c.n_def) break;
                const double *row = dq + (size_t)d * (QF_GROUPS + 1) * MB;
                double v = qf_tree(row + lane, MB);
                if (c.def_add[d]) v = v + row[(size_t)QF_GROUPS * MB + lane];
                const int l = c.def_like[d];
#pragma unroll
                for (int q = 0; q < MAXLIKE; q++)
                    if (q == l) lk[q] = v;
                const_cast<double *>(c.like_terms)[(size_t)l * W + w] = v;
            }
            // GetLogLike (calclike.f90:136-151), target_like's operations in its order
            double like;
            if (oobw[lane]) like = LOGZERO;
            else {
                double main = 0.0;
                bool zero = false;
#pragma unroll
                for (int l = 0; l < MAXLIKE; l++)
                    if (l < c.n_like) {
                        if (lk[l] == LOGZERO) zero = true;
                        main += lk[l];
                    }
                if (zero) like = LOGZERO;
                else {
                    like = main / c.temperature;
                    if (c.has_priors) {
                        double pri = 0.0;
                        for (int i = 0; i < np; i++) pri += zz[(size_t)i * MB + lane];
                        like = like + (pri / 2.0) / c.temperature;
                    }
                }
            }
            bool acc = false;                                     // MetropolisAccept MCMC.f90:119-131
            if (like != LOGZERO) {
                acc = cur > like;
                if (!acc) acc = (double)randexp1(r) > like - cur;
            }
            moved = acc;
            if (acc) {                                            // MoveDone :166-190
                if (mult > 0) nacc += 1;
                mult = 1.0;
                for (int i = 0; i < np; i++) P[(size_t)i * MB] = T[(size_t)i * MB];
                cur = like;
#pragma unroll
                for (int l = 0; l < MAXLIKE; l++)
                    if (l < c.n_like) {
                        ct[l] = lk[l];
                        c.cur_terms[(size_t)l * W + w] = ct[l];
                    }
            } else {
                mult += 1.0;
            }
            c.si[(size_t)R.ACCF * W + w] = acc ? 1 : 0;
            c.si[(size_t)R.NACC * W + w] = nacc;
            c.sd[(size_t)R.L * W + w] = cur;
            c.sd[(size_t)R.M * W + w] = mult;
            if (hist_row) hist_row[(size_t)c.n_used * c.W + w] = cur;
            if (hist_terms) {
#pragma unroll
                for (int l = 0; l < MAXLIKE; l++)
                    if (l < c.n_like) hist_terms[(size_t)l * c.W + w] = ct[l];
            }
        }
        STAMP(3);
        if (PROPOSE) {
            if (!moved)                                           // Trial = CurParams
                for (int i = 0; i < np; i++) T[(size_t)i * MB] = P[(size_t)i * MB];
            // GetProposalFast :283-289: the fast cyclic index over one parameter
            // draws once and always gives it (CyclicIndexRandomizer%Next :75-86)
            (void)ranmar(r);
            // its block's 1 x 1 RotMatrix, drawn at every proposal (:88-102)
            const double r1 = (ranmar(r) - 0.5) >= 0.0 ? 1.0 : -1.0;
            // Propose_r's step length (:122-139), one Gaussian for n = 1
            double rf;
            if (ranmar(r) < 0.33) {
                rf = (double)randexp1(r);
            } else {
                rf = 0.0;
                const double g = gaussian1(r);
                rf += g * g;
                rf = sqrt(rf / 1);
            }
            const double scale = rf * c.propose_scale;
            const double v0 = r1 * scale;
#pragma unroll
            for (int j = 0; j < LEAN_MAXC; j++)                   // UpdateParams :142-149
                if (j < L.nc) {
                    double s = 0.0;
                    s += L.map[j] * v0;
                    T[(size_t)L.chg[j] * MB] += s;
                }
            // the fused pass / bins of this launch poll for the trial calibrations
            if (c.pub_on)
#pragma unroll
                for (int k = 0; k < 2; k++) {
                    const int pc = c.pub_pcal[k];
                    const double v = pc >= 0 ? T[(size_t)pc * MB] : 1.0;
                    __hip_atomic_store(c.calbuf + (size_t)k * W + w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(c.calbuf_next + (size_t)k * W + w,
                                       __longlong_as_double((long long)TP_PIPE_UNSET), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                }
            STAMP(4);
            // DataParams of every likelihood (nuisance_indices)
#pragma unroll
            for (int l = 0; l < MAXLIKE; l++)
#pragma unroll
                for (int q = 0; q < LEAN_MAXQ; q++)
                    if (l < c.n_like && q < L.nn[l])
                        c.like_nuis[l][(size_t)w * L.nn[l] + q] = T[(size_t)L.nuis[l][q] * MB];
            c.sd[(size_t)L.r_row * W + w] = r1;
            c.si[(size_t)(R.CYCLP + 2) * W + w] = 1;
            c.si[(size_t)L.cyc_row * W + w] = 1;
            c.si[(size_t)L.blklp_row * W + w] = 1;
            c.si[(size_t)R.PROT * W + w] = 0;
        }
        c.sd[(size_t)R.C * W + w] = r.c;
        c.sd[(size_t)R.G * W + w] = r.gset;
        c.si[(size_t)R.I97 * W + w] = r.i97;
        c.si[(size_t)R.J97 * W + w] = r.j97;
        c.si[(size_t)R.ISET * W + w] = r.iset;
        ndw[lane] = r.nd < 97 ? r.nd : 97;
        i0w[lane] = i97_0;
    }
    __syncthreads();
    STAMP(12);
    if (!act) return;
    // the thread groups: the ring entries the draws overwrote (positions
    // i97 - 1, i97 - 2, ... mod 97 of the step's first index), P and the
    // trial rows, the history row's parameters
    {
        const int nd = ndw[lane], i0 = i0w[lane];
        for (int t = grp; t < nd; t += NV) {
            int p = i0 - 1 - t;
            if (p < 0) p += 97;
            c.sd[(size_t)(R.U + p) * W + w] = sd[(size_t)(R.U + p) * MB + lane];
        }
    }
    for (int i = grp; i < np; i += NV) {
        if (ACCEPT) c.sd[(size_t)(R.P + i) * W + w] = sp[(size_t)i * MB + lane];
        if (PROPOSE) c.sd[(size_t)(R.T + i) * W + w] = sp[(size_t)(np + i) * MB + lane];
    }
    if (ACCEPT && hist_row) {
#pragma unroll
        for (int u = 0; u < PG; u++) {
            const int i = grp + u * NV;
            if (i < c.n_used) hist_row[(size_t)i * c.W + w] = sp[(size_t)pu[u] * MB + lane];
        }
    }
    STAMP(5);
#ifdef CMAMD_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    STAMP(6);
#endif
}
