// One pass over the walkers' theory rows for the window stages of several
// likelihoods that read the same theory buffer (WinStage, common.h): in the
// headline workload plik_lite's binning (CMB.f90:315-326) and the lensing
// likelihood's bin windows (CMBlikes.f90:1230-1256) both read TT, TE and EE;
// run as one pass, each walker's rows leave HBM once instead of twice.
#pragma once

#include <map>

#include "common.h"

namespace cmamd {

static constexpr int TP_MAXOUT = 2;    // likelihoods per pass
static constexpr int TP_CHUNK = 64;    // l per weight chunk
static constexpr int TP_MAXCOL = 64;   // columns per work item (four 16-column MFMA blocks)
#ifndef CMAMD_TP_MAXL
#define CMAMD_TP_MAXL 352
#endif
// l per work item, unless overlapping columns force more (at most
// TP_MAXSTEP * 32 - 1 in any case).  Round 2 (the standalone pass alone):
// 288 (9 steps), 22.7 us against 24.0 (256), 23.2 (272), 23.3 (300), 23.6 (320),
// 24.9 (384).  Round 6, with the pass inside the unified step launch (fewer,
// longer units beside the quadratic form) and the two-step weight prefetch:
// 352 (11 steps), middle launch 33.2-33.7 -> 32.0-32.5 us and the drag step
// 407-413 -> 399-405 us, against 192 / 224 / 256 / 320 / 336 / 368 / 384 / 416 /
// 448 (34.2 / 34.6 / 33.2 / 33.2 / 32.6-32.9 / 32.9-33.0 / 32.6-32.7 / 33.3 / 34.0 us
// a launch; tools/gpu_r6j.sh; the drag's pair pass 165-180 us a drag step at
// 320-368 against 152-153 at 352); at 480
// some l range needs more than TP_MAXCOL columns and the fused pass is not built
static constexpr int TP_MAXL = CMAMD_TP_MAXL;

struct TPOut {            // a stage's output for one launch
    int kind;             // WinStage::kind
    int cal_index;        // calibration parameter index in nuis (-1: none)
    int ld;               // kind 1: row stride of out
    int pad;
    double *out;          // kind 0: [row][W]; kind 1: [W][ld]
    const double *X;      // kind 1
    const double *nuis;   // [W][ld_nuis]
    long long ld_nuis;
};

static constexpr int TP_MAXSTEP = 16;
// a calibration slot not yet published in this launch (a NaN payload no
// calibration takes; compared by bits)
static constexpr unsigned long long TP_PIPE_UNSET = 0x7ff4c0ffee0dd00dull;
// published instead of a calibration when the walker's proposal waits on a new
// rotation (rot_kernel finishes it after the launch; the bin co-run)
static constexpr unsigned long long TP_PIPE_ROT = 0x7ff4c0ffee0dd00eull;   // 32-l steps per work item (the active-block mask)

struct TPItem {           // one workgroup's l range of one theory field, with <= 64 columns
    int field, l0, l1, nch, ncol, cdesc;
    int nst;              // 32-l steps: ceil((l1 - l0 + 1) / 32) (<= 2 nch)
    int nsb;              // 16-slot MFMA blocks in use (slots are reused: TheoryPass::build)
    int soff;             // first of its steps in TPDev::emit / cmap
    long long woff;       // weights [nch][nsb][16 slots][TP_CHUNK], zero padded
    unsigned long long act;   // bit 4 step + block: the block has a nonzero weight in the step
};

struct TPCol {
    int out, row, cal, pad;
};

struct TPDev {
    const TPItem *items;
    const int2 *units;    // per block: (item, walker tile), item -1: no work
    const TPCol *cols;
    const double *w;
    const unsigned long long *emit;   // per item step: slots whose column ends there
    const unsigned char *cmap;        // per item step, [64] slots: the item's column index (255: none)
    int nitem;
    int nblk;             // block table entries (units, including empty ones)
    int tile_off;         // the units' walker tiles start here (0: the pass over every walker)
    TPOut out[TP_MAXOUT];
};

class TheoryPass {
  public:
    // pack the stages' columns into work items (no column split between two);
    // false when some l range needs more than TP_MAXCOL columns
    bool build(const std::vector<WinStage> &stages);
    void launch(const double *dl, long long ld_field, long long ld_walker, const TPOut *outs, int W,
                hipStream_t stream);
    // the pass over two theory sets in one launch (theory_window_pair; both
    // vec_ok), zeroing nz tickets at za / zb for the quadratic form after it
    // (dlb null: set a alone)
    void launch_pair(const double *dla, long long lfa, long long lwa, const TPOut *oa, unsigned int *za,
                     const double *dlb, long long lfb, long long lwb, const TPOut *ob, unsigned int *zb, int nz, int W,
                     hipStream_t stream);
    // The vectorised kernel applies (16-byte aligned rows, at most two MFMA
    // blocks per item): the form the sampler's pipelined steps run
    bool vec_ok(const double *dl, long long ld_field, long long ld_walker) const;
    // its arguments and block count for W walkers (theorypass_body.h)
    TPDev dev_args(const TPOut *outs, int W);
    int n_blocks() const { return nblk; }

    int n_items() const { return (int)items.size(); }
    const TPItem &item(int k) const { return items[k]; }
    int n_stages() const { return nstage; }

  private:
    // the block table for `tiles` walker tiles (plan_units)
    void plan_units(int tiles);
    std::vector<TPItem> items;
    DevBuf d_items, d_cols, d_w, d_units, d_emit, d_cmap;
    int nstage = 0;
    int unit_tiles = -1, nblk = 0, max_nsb = 0, per_round = 0;
};

}  // namespace cmamd
