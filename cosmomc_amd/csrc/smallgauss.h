// Chi^2 of a small gaussian CMBlikes dataset (nX <= 64 bandpowers: Planck
// lensing's 9, SPT-SZ's 47) from its window stage's partial rows --
// CMBLikes_LogLike's binned spectra with the linear correction, bigX = C - Chat
// and Matrix_QuadForm (CMBlikes.f90:1183-1225), plus the log-calibration prior
// (:1222-1223).  Shared by the standalone cmbl_gauss_small_kernel
// (cmblikes.hip) and the sampler's accepting mh_kernel (sampler.hip), which
// takes the chi^2 over in the fast steps, so both sum in the one order defined
// here: a task is <= 8 partial rows summed in row order; an element sums its
// tasks in order; z_i = x_i (M x)_i with j in order; chi^2 = sum of z_i in i
// order.  The caller lays out the threads as NG groups of WT walkers and puts
// a barrier between the phases.
#pragma once

#include <hip/hip_runtime.h>

namespace cmamd {

static constexpr int SG_ROWS = 8;            // partial rows per task

struct SmallGaussDev {
    int nE, nX, ntask, has_corr, cal_index;  // cal_index: in the nuisance vector, -1 none
    double log_cal_prior;                    // > 0: add (ln cal / prior)^2
    const int *trow;                         // [ntask][SG_ROWS] partial rows of each task, -1 padded
    const int *e_main_t, *e_corr_t;          // [nE + 1] task ranges per element (main windows, linear correction)
    const int *e_to_x;                       // [nE] index into bigX, or -1
    const double *e_main_const, *e_corr_const, *fidcorr, *chat;   // [nE]
    const double *M;                         // [nX][nX] inverse bandpower covariance
};

// phase 1: tasks t = g, g + NG, ... of walker w (partial row stride ldp) into tp[t][WT]
template <int WT, int NG>
__device__ inline void sg_tasks(const SmallGaussDev &c, const double *__restrict__ partial, long long ldp, int w,
                                bool act, int g, int wl, double *tp)
{
    for (int t = g; t < c.ntask; t += NG) {
        const int4 ra = *reinterpret_cast<const int4 *>(c.trow + SG_ROWS * t);
        const int4 rb = *reinterpret_cast<const int4 *>(c.trow + SG_ROWS * t + 4);
        const int r[SG_ROWS] = {ra.x, ra.y, ra.z, ra.w, rb.x, rb.y, rb.z, rb.w};
        double v[SG_ROWS];
#pragma unroll
        for (int u = 0; u < SG_ROWS; u++) v[u] = (act && r[u] >= 0) ? partial[(long long)r[u] * ldp + w] : 0.0;
        double s = 0.0;
#pragma unroll
        for (int u = 0; u < SG_ROWS; u++) s += v[u];
        tp[t * WT + wl] = s;
    }
}

// phase 2: element e = g, g + NG, ...: its binned spectrum minus Chat into xs[ix][WT]
template <int WT, int NG>
__device__ inline void sg_elems(const SmallGaussDev &c, int g, int wl, const double *tp, double *xs)
{
    for (int e = g; e < c.nE; e += NG) {
        const int ix = c.e_to_x[e];
        if (ix < 0) continue;
        double s = c.e_main_const[e];
        for (int t = c.e_main_t[e]; t < c.e_main_t[e + 1]; t++) s += tp[t * WT + wl];
        if (c.has_corr) {
            double cs = c.e_corr_const[e];
            for (int t = c.e_corr_t[e]; t < c.e_corr_t[e + 1]; t++) cs += tp[t * WT + wl];
            s = s + (cs - c.fidcorr[e]);
        }
        xs[ix * WT + wl] = s - c.chat[e];
    }
}

// phase 3: z_i = x_i (M x)_i for rows i = g, g + NG, ... into z[i][WT]
template <int WT, int NG>
__device__ inline void sg_rows(const SmallGaussDev &c, const double *M, int g, int wl, const double *xs, double *z)
{
    for (int i = g; i < c.nX; i += NG) {
        double y = 0.0;
        for (int j = 0; j < c.nX; j++) y += M[i * c.nX + j] * xs[j * WT + wl];
        z[i * WT + wl] = xs[i * WT + wl] * y;
    }
}

// phase 4 (one thread per walker): -lnL = (sum_i z_i + calibration prior) / 2
template <int WT>
__device__ inline double sg_final(const SmallGaussDev &c, int wl, const double *z, double cal)
{
    double chisq = 0.0;
    for (int i = 0; i < c.nX; i++) chisq += z[i * WT + wl];
    if (c.log_cal_prior > 0 && c.cal_index >= 0) {
        const double t = log(cal) / c.log_cal_prior;
        chisq = chisq + t * t;
    }
    return chisq / 2;
}

}  // namespace cmamd
