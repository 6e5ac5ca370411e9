// Small gaussian CMBlikes chi^2 (nX <= 64 bandpowers, e.g. Planck lensing 9,
// SPT-SZ 47): binned spectra, bigX = C - Chat and chi^2 = bigX^T C^-1 bigX in
// one workgroup body (CMBlikes.f90:1183-1225; Matrix_QuadForm as row sums
// y = M x, then x.y).  Shared by cmbl_gauss_small_kernel (cmblikes.hip) and by
// the deferred quadratic form's launch (quadform.hip, quadform_corun), where
// its workgroups run beside the quadratic form's instead of in a launch of
// their own.  The arguments are SmallGaussLaunch (common.h).
//
// Workgroup = WT walkers x 256 / WT thread groups.  The partial rows of every
// element are cut into tasks of <= 8 rows (host); groups take tasks
// round-robin with all loads of a task in flight, then combine them per
// element in task order (deterministic), then split the rows of M.  Every
// table load is issued at the start, beside the others: the partial loads
// wait on one table level (the task's rows), nothing after them on any.
#pragma once

#include "common.h"
#include "divrn.h"

namespace cmamd {

static constexpr int SMALL_NX = 64;
static constexpr int SMALL_WT = 4;          // walkers per workgroup (measured: 7.1 / 8.0 / 9.8 / 13.9 us for 4 / 2 / 8 / 16)
static constexpr int SMALL_MAXTASK = 256;   // tasks per dataset

// LDS of one workgroup body: tp[SMALL_MAXTASK][WT], xs[SMALL_NX][WT],
// red[256 / WT][WT], M[SMALL_NX][SMALL_NX]
template <int WT> constexpr int small_gauss_lds_doubles() {
    return SMALL_MAXTASK * WT + SMALL_NX * WT + 256 + SMALL_NX * SMALL_NX;
}
// the same for an nX-bandpower dataset (M takes nX^2 doubles)
template <int WT> constexpr int small_gauss_lds_doubles(int nX) {
    return SMALL_MAXTASK * WT + SMALL_NX * WT + 256 + nX * nX;
}

// Walker group of workgroup lb among ng (a launch gives the role 8 ceil(ng / 8)
// workgroups, from a multiple of 8): workgroup b runs on XCD b % 8, so with
// lb % 8 the XCD each XCD takes a contiguous range of groups and a partial
// row's 128-byte lines (16 walkers) are read by one L2 instead of four.
// Groups >= ng: none.
__device__ __forceinline__ int small_gauss_group(int lb, int ng)
{
    return (lb & 7) * ((ng + 7) >> 3) + (lb >> 3);
}
__host__ __device__ inline int small_gauss_blocks(int ng) { return (ng + 7) & ~7; }

// RAWCAL: partial rows are raw window sums; rows flagged in a.row_cal are
// divided by the walker's cal^2 as they are loaded (SmallGaussLaunch)
// SIGNAL: -lnL is stored agent-scope (write-through) for a consumer in the
// same launch (the sampler's unified step launch)
// TPF: tasks whose loads a thread group has in flight at once (the same sums,
// task by task; the folded chi^2 of the unified launch, which is latency on the
// Metropolis workgroups' path, takes 2)
template <int WT, bool RAWCAL = false, bool SIGNAL = false, int TPF = 1>
__device__ __forceinline__ void small_gauss_body(const SmallGaussLaunch &a, double *lds, int blk)
{
    constexpr int NG = 256 / WT;             // thread groups of WT walkers
    double *tp = lds;                        // [SMALL_MAXTASK][WT]
    double *xs = tp + SMALL_MAXTASK * WT;    // [SMALL_NX][WT]
    double *red = xs + SMALL_NX * WT;        // [NG][WT]
    double *Msh = red + NG * WT;             // [nX][nX]
    const SmallGaussDev &c = a.d;
    const int W = a.W;
    const int wl = threadIdx.x % WT, g = threadIdx.x / WT;
    const int w = blk * WT + wl;
    const int Wc = c.wcount ? min(W, *c.wcount) : W;
    if (blk * WT >= Wc) return;
    for (int i = threadIdx.x; i < c.nX * c.nX; i += 256) Msh[i] = a.M[i];   // in flight with the partial loads
    const bool act = w < Wc;
    const bool calp = c.log_cal_prior > 0 && c.cal_index >= 0;
    const double cal = (g == 0 && act && calp) ? a.nuis[(long long)w * a.ld_nuis + c.cal_index] : 1.0;   // likewise
    double c2 = 1.0, rc2 = 1.0;   // RAWCAL: the stage calibration's square, as the pass's emit forms it
    if (RAWCAL && act && a.stage_cal >= 0) {
        const double cl = a.nuis[(long long)w * a.ld_nuis + a.stage_cal];
        c2 = cl * cl;
        rc2 = 1.0 / c2;
    }
    struct Elem { int ix, m0, m1, c0, c1; double mc, cc, fc, ch; };
    auto elem = [&](int e) {   // element e's table entries
        Elem q{c.e_to_x[e], c.e_main_t[e], c.e_main_t[e + 1], 0, 0, c.e_main_const[e], 0.0, 0.0, c.chat[e]};
        if (c.has_corr) {
            q.c0 = c.e_corr_t[e];
            q.c1 = c.e_corr_t[e + 1];
            q.cc = c.e_corr_const[e];
            q.fc = c.fidcorr[e];
        }
        return q;
    };
    Elem e0{-1, 0, 0, 0, 0, 0.0, 0.0, 0.0, 0.0};
    if (g < c.nE) e0 = elem(g);   // this group's first element, in flight with the partials
    for (int t0 = g; t0 < c.ntask; t0 += NG * TPF) {
        int r[TPF][8];
        double v[TPF][8];
#pragma unroll
        for (int p = 0; p < TPF; p++) {
            const int t = t0 + p * NG;
            const bool ok = t < c.ntask;
            const int4 ra = ok ? *reinterpret_cast<const int4 *>(c.trow + 8 * t) : make_int4(-1, -1, -1, -1);
            const int4 rb = ok ? *reinterpret_cast<const int4 *>(c.trow + 8 * t + 4) : make_int4(-1, -1, -1, -1);
            r[p][0] = ra.x; r[p][1] = ra.y; r[p][2] = ra.z; r[p][3] = ra.w;
            r[p][4] = rb.x; r[p][5] = rb.y; r[p][6] = rb.z; r[p][7] = rb.w;
        }
#pragma unroll
        for (int p = 0; p < TPF; p++)
#pragma unroll
            for (int u = 0; u < 8; u++) v[p][u] = (act && r[p][u] >= 0) ? a.partial[(long long)r[p][u] * W + w] : 0.0;
#pragma unroll
        for (int p = 0; p < TPF; p++) {
            const int t = t0 + p * NG;
            if (t >= c.ntask) break;
            if (RAWCAL)
#pragma unroll
                for (int u = 0; u < 8; u++)
                    if (r[p][u] >= 0 && a.row_cal[r[p][u]]) v[p][u] = div_rn(v[p][u], c2, rc2);   // = v / c2
            double s = 0.0;
#pragma unroll
            for (int u = 0; u < 8; u++) s += v[p][u];
            tp[t * WT + wl] = s;
        }
    }
    __syncthreads();
    for (int e = g; e < c.nE; e += NG) {
        const Elem q = e == g ? e0 : elem(e);
        if (q.ix < 0) continue;
        double s = q.mc;
        for (int t = q.m0; t < q.m1; t++) s += tp[t * WT + wl];
        if (c.has_corr) {
            double cs = q.cc;
            for (int t = q.c0; t < q.c1; t++) cs += tp[t * WT + wl];
            s = s + (cs - q.fc);
        }
        xs[q.ix * WT + wl] = s - q.ch;
    }
    __syncthreads();
    double part = 0.0;
    for (int i = g; i < c.nX; i += NG) {
        double y = 0.0;
        for (int j = 0; j < c.nX; j++) y += Msh[i * c.nX + j] * xs[j * WT + wl];
        part += xs[i * WT + wl] * y;
    }
    red[g * WT + wl] = part;
    __syncthreads();
    if (g == 0 && act) {
        double chisq = 0.0;
        for (int k = 0; k < NG; k++) chisq += red[k * WT + wl];
        if (calp) {
            const double t = log(cal) / c.log_cal_prior;
            chisq = chisq + t * t;
        }
        if (SIGNAL)
            __hip_atomic_store(a.out + w, chisq / 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else
            a.out[w] = chisq / 2;
    }
}

}  // namespace cmamd
