// Internal sampler state shared by sampler.hip and api.cpp.
#pragma once

#include "common.h"

namespace cmamd {

struct DevCfg {
    int W, np, n_used, nblocks, slow_n, fast_n, all_n, oversample_fast;
    double propose_scale, temperature;
    // shared proposer tables
    const int *blk_n, *blk_nchanged, *blk_changed_off, *blk_map_off, *blk_R_off;
    const int *changed;             // 0-based parameter indices
    const double *mapping;          // per block nchanged x n, row-major
    const int *proposer_for_index;  // all_n, 1-based block
    const double *pmin, *pmax, *prior_mean, *prior_std;
    int has_priors;
    // test gaussian
    int test_like;
    const int *params_used;         // n_used, 0-based
    const double *test_covinv;      // n_used^2
    const double *center;           // np
    // per-walker state (SoA)
    double *rng_u;                  // [97][W]
    double *rng_c, *rng_gset;       // [W]
    int *rng_i97, *rng_j97, *rng_iset;
    int R_total;                    // sum n_b^2
    double *R;                      // [R_total][W]
    int *blk_loopix;                // [nblocks][W]
    int *cyc;                       // [all_n + slow_n + fast_n][W] index permutations
    int *cyc_loopix;                // [3][W]: all, slow, fast
    int *fast_ix;                   // [W]
    double *P, *trial;              // [np][W]
    double *cur_like, *mult;        // [W]
    int *num_accept;                // [W]
    int n_like;
    const double *like_terms;       // [n_like][W] -lnL of each likelihood at trial
    int like_nuis0[8], like_nn[8];  // nuisance slice of each likelihood (0-based start, count)
    double *like_nuis[8];           // [W][like_nn] DataParams buffers written by mh_kernel
    int max_blk;                    // largest proposal block
};

static constexpr int MAXLIKE = 8;

struct LikeSlot {
    cmbl_t *like;
    int nuis0;   // 0-based
    const double *dl;
    long long ld_field, ld_walker;
};

}  // namespace cmamd

struct cmbs {
    cmamd::DevCfg dc{};
    int W = 0, np = 0, n_used = 0;
    std::vector<int> params_used, blk_n, blk_params;
    int slow_block_max = 0;
    std::string last_error;
    // device buffers
    cmamd::DevBuf tables, state, covinv, center, like_terms, ws, hist;
    cmamd::DevBuf nuis_bufs[cmamd::MAXLIKE];
    std::vector<cmamd::LikeSlot> likes;
    // host copies of the proposer structure
    std::vector<int> indices, proposer_for_index, blk_start, blk_nchanged, used_params_changed_all;
    std::vector<int> blk_changed_off, blk_map_off, blk_R_off, changed;
    int all_n = 0, slow_n = 0, fast_n = 0, nblocks = 0, R_total = 0, map_total = 0;
    int hist_cap = 0, hist_count = 0;
    bool started = false;
};

