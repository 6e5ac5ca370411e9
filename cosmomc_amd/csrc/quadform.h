// Batched symmetric quadratic form  q_w = x_w^T M x_w / 2  for a fixed SPD
// (inverse-covariance) matrix M and W walker vectors x_w, on the f64 MFMA.
// Shared by every likelihood whose -lnL ends in Matrix_QuadForm
// (source/Matrix_utils_new.f90:2033-2047): plik_lite (CMB.f90:327) and
// CMBlikes (CMBlikes.f90:1220).
//
// Layout: the producer kernel writes x into the workspace as rows
// x[w][Np] (Np = n rounded up to 64, zero-padded) and zeroes the
// arrival counters (counters(ws)) before launch() runs on the same stream.
#pragma once

#include <map>
#include <vector>

#include "common.h"

namespace cmamd {

static constexpr int QF_TILE = 64;   // M block edge and walker tile

struct QFItem {   // one workgroup's share: row block I x column blocks J0 .. J0+nJ-1 (all >= I)
    int I, J0, nJ, pad;
};
static constexpr int QF_MAXKB = 5;   // column blocks per item at most (QuadForm::choose_kb)

// Split-K combine, one fixed order shared by the in-launch reducer and by a
// deferred consumer (the sampler's mh_kernel), so both give the same bits:
// partials p[tile][k][64]; group g sums k = g, g+16, ... ascending from 0.0
// (loads issued 8 at a time); the 16 group sums meet in a fixed pairwise
// tree; then + addend.
static constexpr int QF_GROUPS = 16;
static constexpr int QF_GROUP_DEPTH = 8;

__device__ inline double qf_group_sum(const double *tile_part, int n_items, int g, int lane) {
    double r = 0.0;
    for (int k0 = g; k0 < n_items; k0 += QF_GROUPS * QF_GROUP_DEPTH) {
        double v[QF_GROUP_DEPTH];
#pragma unroll
        for (int j = 0; j < QF_GROUP_DEPTH; j++) {      // every load in flight before the first add
            const int k = k0 + QF_GROUPS * j;
            v[j] = (k < n_items) ? tile_part[(size_t)k * QF_TILE + lane] : 0.0;
        }
#pragma unroll
        for (int j = 0; j < QF_GROUP_DEPTH; j++) r += v[j];
    }
    return r;
}

// r[g * stride]: the 16 group sums
__device__ inline double qf_tree(const double *r, int stride) {
    double a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = r[i * stride] + r[(i + 8) * stride];
#pragma unroll
    for (int i = 0; i < 4; i++) a[i] = a[i] + a[i + 4];
    a[0] = a[0] + a[2];
    a[1] = a[1] + a[3];
    return a[0] + a[1];
}


class QuadForm {
  public:
    // M: n x n row-major symmetric
    void init(const std::vector<double> &M, int n);
    int n = 0, Np = 0;
    static int wpad(int W) { return (W + QF_TILE - 1) / QF_TILE * QF_TILE; }
    size_t workspace_size(int W) const;
    double *x_rows(void *ws) const { return static_cast<double *>(ws); }
    unsigned int *counters(void *ws, int W) const;
    int n_counters(int W) const { return wpad(W) / QF_TILE; }
    // out[w] = x_w^T M x_w / 2 + (addend ? addend[w] : 0)
    // wcount (device int, or null): only walkers [0, *wcount) are live
    void launch(int W, void *ws, const double *addend, double *out, hipStream_t stream, const char *prof_name,
                const int *wcount = nullptr);
    // the same launch without the combine: the workgroups store their partials
    // and exit; the returned descriptor tells a later kernel how to finish
    // co: a small gaussian chi^2 whose workgroups run in the same launch
    // (quadform_corun), timed as co_prof_name
    QFDeferred launch_deferred(int W, void *ws, const double *addend, hipStream_t stream, const char *prof_name,
                               const SmallGaussLaunch *co = nullptr, const char *co_prof_name = nullptr);

    // the deferred launch's operands for a launch that forms the rows itself
    // (X: the data vector the rows are X - S / cal^2 of)
    QFSource source(int W, void *ws, const double *X);

  private:
    static constexpr int MAXKB = QF_MAXKB;
    int nblk = 0;
    DevBuf d_ct;
    DevBuf d_items[MAXKB + 1];
    std::vector<QFItem> items[MAXKB + 1];
    std::map<int, int> kb_for_tiles;
    size_t nmax_items() const;
    int choose_kb(int tiles);
};

// Two in-launch-combined quadratic forms (QFSource with delta / counters; the
// tickets zero at launch) and optionally two small chi^2s in one launch
// (quadform_pair_ticket): out_a / out_b get -lnL of the two walker sets.
// qb / gb null: set a alone (its quadratic form and chi^2 in one launch)
void launch_qf_pair(const QFSource &qa, double *out_a, const QFSource *qb, double *out_b, int W,
                    const SmallGaussLaunch *ga, const SmallGaussLaunch *gb, hipStream_t stream, const char *prof_name);

// host symmetric-matrix helpers (row-major)
void spd_inverse(std::vector<double> &A, int n);                       // Matrix_Inverse
void sym_eigen(std::vector<double> A, int n, std::vector<double> &evals,
               std::vector<double> &evecs);                            // Matrix_Diagonalize
void sym_power(std::vector<double> &A, int n, double pw);             // Matrix_Root

}  // namespace cmamd
