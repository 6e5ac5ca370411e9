// The sampler's unified step launch (sampler.hip mh_step_kernel): one launch
// per fast step runs, side by side,
//   * plik_lite's deferred quadratic form of step k, its operand rows formed
//     in registers from the raw bin sums of step k and the walkers' step-k
//     calibrations (Delta = X - S / cal^2, the pass's own emit operations),
//   * the small gaussian chi^2 of the fused CMBlikes dataset (Planck lensing)
//     of step k, its raw partial rows calibrated as they are loaded,
//   * the fused window pass over every walker's theory for step k + 1, which
//     stores raw sums (no calibration: those of step k + 1 are not proposed
//     yet) into the other half of a two-half buffer, and
//   * the Metropolis workgroups, which wait for their walker tile's quadratic
//     form and chi^2, accept step k and propose step k + 1.
// The pass is HBM-bound and the quadratic form MFMA / L2-bound, so they share
// the CUs instead of following each other.
#pragma once

#include <vector>

#include "common.h"
#include "theorypass.h"

namespace cmamd {

struct QFSArgs {             // the quadratic form from raw sums (QFSource + the step's rows)
    QFSource src;
    const double *S;         // [Wp][Np] raw bin sums (padding rows and columns zero)
    const double *nuis;      // [W][ld_nuis] the walkers' step-k nuisance values
    long long ld_nuis;
    int cal_index;           // cal in nuis (-1: none)
    int W;
};

struct StepTail {
    QFSArgs q;
    int nq = 0;              // quadratic-form workgroups (n_items x tiles), 0: none
    SmallGaussLaunch g{};
    int ng = 0;              // chi^2 workgroups, 0: none
    int fold_g = 0;          // the chi^2 runs inside the Metropolis workgroups (16 walkers each), not as rows
    int qf_ahead = 0;        // middle launches: the quadratic form's two-step-ahead form (qfs_body_nj)
    int fold_late_prio = 0;  // the Metropolis workgroups take issue priority only after the folded chi^2
    int qf_prio = 0;         // the quadratic-form waves at issue priority 2
    int fold_tpf = 1;        // the folded chi^2's tasks in flight per thread group
    TPDev tp{};              // the raw pass (tp.out[*].out: the raw-sum buffers it writes)
    const double *dl = nullptr;
    long long ld_field = 0, ld_walker = 0;
    int np = 0;              // pass workgroups (TheoryPass::n_blocks), 0: none
    int W = 0;
};

// Workgroup roles by rows of 8 (block b runs on XCD b % 8, so each role's own
// block numbering keeps the XCD placement its body assumes: qf_place,
// TheoryPass::plan_units): row k is role rows[k].x's rows[k].y-th row.  The nm
// Metropolis workgroups come last.
enum { TAIL_QF = 0, TAIL_GAUSS = 1, TAIL_PASS = 2, TAIL_MH = 3 };
std::vector<int2> tail_rows(int nq, int ng, int np, int nm);

// the launch's workgroup rows for its role counts (owned by the caller)
struct StepTailPlan {
    DevBuf d_rows;
    int key[3] = {-1, -1, -1};
    int nrows = 0;
};


}  // namespace cmamd
