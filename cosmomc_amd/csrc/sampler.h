// Internal sampler state shared by sampler.hip and api.cpp.
#pragma once

#include "common.h"
#include "steptail.h"
#include "theorypass.h"

namespace cmamd {

static constexpr int MAXLIKE = 8;
static constexpr int MAXGROUPS = 8;
static constexpr int MAXDEF = 2;        // likelihoods whose split-K combine mh_kernel can take over

// Per-walker state is two row-major SoA arrays in HBM, sd[ND][W] (doubles)
// and si[NI][W] (ints): row r of walker w at sd[r*W + w].  mh_kernel copies
// a 64-walker column block of every row into LDS with independent coalesced
// loads, runs the sequential chain logic out of LDS, and writes it back.
struct Rows {
    // double rows
    int U = 0;          // 97 rows: RANMAR u(1:97)
    int C = 97;         // RANMAR c
    int G = 98;         // Gaussian1 saved deviate gset
    int R = 100;        // R_rows rows (R_total rounded up to even): per-block random rotations
                        //   (row j col i of block b at R + off_b + j*n+i); row 99 is padding
    int RR;             // R_rows
    int P, T, L, M;     // np rows current point, np rows trial, cur_like, mult
    int ND;             // even: rows are moved in pairs (16-byte LDS-DMA pieces)
    // int rows
    int I97 = 0, J97 = 1, ISET = 2, FASTIX = 3, NACC = 4;
    int CYCLP = 5;      // 3 rows: All, Slow, Fast CyclicIndexRandomizer%loopix
    int BLKLP = 8;      // nblocks rows: RandDirectionProposer%loopix
    int ACCF;           // 1 if the last accept of this walker moved it (theory swap for slow steps)
    int PROT;           // b + 1 while block b's new random rotation is pending for rot_kernel, else 0
    int CYC;            // multiple of 4; all_n + slow_n + fast_n rows: the three index permutations
                        //   (last, so an LDS image without them is the prefix [0, CYC))
    int NI;             // multiple of 4: rows are moved four at a time
};

// Shared read-only tables (copied to LDS by every mh_kernel block).
struct TabLayout {
    // int table offsets (ints)
    int blk_n, blk_nchanged, blk_changed_off, blk_map_off, blk_R_off, changed, pfi, params_used, n_int;
    // double table offsets (doubles)
    int mapping, pmin, pmax, pmean, pstd, lin_w, lin_m, lin_s, covinv, center, n_dbl;
};

// The lean Metropolis chain (mhlean.h): fast-only steps whose only fast
// parameter is a one-parameter block (the headline's calPlanck).  The host
// resolves the block's rows, changed parameters, mapping column and the
// likelihoods' nuisance indices into this struct per launch, so the chain
// reads them from kernel arguments instead of LDS table lookups.
static constexpr int LEAN_MAXC = 8;     // changed parameters of the block
static constexpr int LEAN_MAXQ = 4;     // nuisance indices per likelihood
// (every array below is indexed by compile-time indices only: an index known
// only at run time would make the compiler copy the kernel arguments to scratch)
struct LeanCfg {
    int on;                             // this launch runs mh_lean
    int nc;                             // changed parameters of the fast block
    int r_row, cyc_row, blklp_row;      // its rotation row (sd), cyclic-index row, loop-index row (si)
    int chg[LEAN_MAXC];                 // changed parameters (0-based)
    double map[LEAN_MAXC];              // the block's mapping column (UpdateParams, propose.f90:142-149)
    int nn[MAXLIKE];                    // likelihood l's nuisance parameters
    int nuis[MAXLIKE][LEAN_MAXQ];       // their 0-based parameter indices
};

struct DevCfg {
    LeanCfg lean;           // first: read in one batch at the start of the lean chain
    int W, np, n_used, nblocks, slow_n, fast_n, all_n, oversample_fast, max_blk, R_total;
    int ld;                 // row stride of sd / si / like_terms: W rounded up to 64
    double propose_scale, temperature;
    int has_priors, test_like, n_lin;
    int rot_defer;          // mh_kernel leaves new rotations of blocks >= ROT_DEFER_MIN to rot_kernel
    int *rot_list;          // [ld] walkers whose rotation is pending, listed per 64-walker-aligned range from its start
    int *rot_cnt;           // [ld / 64][2] list lengths; a proposing launch appends to rot_par, zeroes the other
    int rot_par;            // set per launch
    int rot_serial;         // debug: 1 every rotation by the serial path, 2 parallel without speculative lanes
    Rows rows;
    TabLayout tl;
    const int *tab_i;       // [tl.n_int] (allocation padded to a multiple of 64 words)
    const double *tab_d;    // [tl.n_dbl] (allocation padded to a multiple of 32 doubles)
    double *sd;             // [ND][ld]
    int *si;                // [NI][ld]
    int stage_R;            // R rows staged in LDS (else read in place, stride W)
    int pre_blk;            // the only fast block (0-based; -1: several, or one parameter wide): with R
                            //   in place, fast-only proposals have its next column fetched beside the image
    int pre_lp;             // pre_blk's loop index for every walker of this launch when the host knows it
                            //   (rot_may_pend), else -1: the column's loads then go out with the image's
    int pre_off, pre_n;     // pre_blk's R offset and width
    int stage_cyc;          // CYC rows + RandIndices scratch in LDS (else in place / itmp_g)
    int stage_cov;          // test-Gaussian covinv + center tables in LDS (else read from tab_d)
    int *itmp_g;            // [all_n][ld] RandIndices scratch when !stage_cyc
    int tq_rows;            // LDS scratch rows for the multi-wave test-Gaussian / mapping products
    int n_like;
    const double *like_terms;       // [n_like (even)][ld] -lnL of each likelihood at the trial point
    double *cur_terms;              // [n_like][ld] -lnL of each likelihood at the current point
                                    //   (TCalculationAtParamPoint%Likelihoods, for chi2_* output)
    int like_nidx[MAXLIKE], like_nn[MAXLIKE];   // offset in tab_i of each likelihood's nuisance_indices
                                                //   (0-based indices into P), and their count
    double *like_nuis[MAXLIKE];     // [W][like_nn] DataParams buffers written by mh_kernel
    // per-likelihood change mask (LogLikeWithTheorySet, calclike.f90:374-386): a
    // likelihood is re-evaluated only for walkers whose trial moved one of its
    // dependent parameters (its nuisance parameters and every theory parameter);
    // the others keep their current-point term (TCalculationAtParamPoint%Likelihoods)
    unsigned long long like_dep[MAXLIKE];   // dependent-parameter bits (0-based parameter index)
    int mask_on;                            // this launch uses the mask (set per launch)
    int *like_flag;                         // [n_like][ld]: 0 unchanged, else 1 (dense) or compact slot + 1 (sparse)
    const double *like_out[MAXLIKE];        // sparse likelihoods: terms by compact slot; null = dense (like_terms)
    // deferred quadratic-form combines (QFDeferred): the accepting mh_kernel
    // finishes these likelihoods' -lnL from the split-K partials the step's
    // evaluation left (one kernel boundary and no in-launch hand-off)
    int def_cap;                            // LDS room: group-sum rows for this many likelihoods
    int n_def;                              // this launch: deferred likelihoods to finish (set per launch)
    int def_like[MAXDEF], def_items[MAXDEF];
    const double *def_part[MAXDEF];         // [tiles][def_items][64]
    const double *def_add[MAXDEF];          // [W] or null
    // bin co-run (mh_bin_kernel): a proposing launch publishes the trial
    // calibrations of every walker into calbuf (this launch's half) and resets
    // the other half to PIPE_UNSET for the next launch; the bin workgroups
    // poll for their walkers' values
    int pub_on;                             // set per launch
    int pub_pcal[2];                        // the stages' calibration parameters (0-based, -1: none)
    double *calbuf;                         // [2 stages][ld], this launch's half
    double *calbuf_next;                    // the next launch's half
    // bin co-run (mh_bin_kernel): rot_kernel forms the Delta rows of the
    // walkers it finishes from the co-run's raw sums (bin_on: set per launch)
    int bin_on, bin_nused, bin_Np, bin_cal;  // bin_cal: plik's calibration among its nuisances
    const double *bin_S, *bin_X;            // [wpad(W)][Np] raw sums; [Np] data vector
    double *bin_delta;                      // [wpad(W)][Np] plik's Delta rows
};

// The unified step launch (sampler.hip mh_step_kernel): its
// Metropolis workgroups wait for their walker tile's quadratic-form and
// chi^2 workgroups of the same launch, which arrive on a per-tile counter
// after their outputs are stored write-through.  The counters only grow: a
// tile is complete in this launch's epoch e when its count reaches e x (its
// producers per launch).
struct TailWait {
    unsigned int *cnt;       // [tiles] arrivals
    unsigned int epoch;      // launches with producers so far, this one included
    unsigned int epoch_g;    // of them, those whose chi^2 ran as workgroups of its own (not folded)
    int nq_items;            // quadratic-form workgroups per tile
    int ng, gwt;             // chi^2 workgroups (of an unfolded launch) and walkers per chi^2 workgroup
    int *status;             // CMBL_STATUS_PIPE_WAIT when a wait gives up
    int nosignal;            // debug: the producers never arrive (the give-up test)
    int stamp_slot;          // instrumented builds: the stamp buffer (0 middle launches, 1 the last)
    int ntiles;              // counters (the first launch of a call zeroes them)
};

struct LikeSlot {
    cmbl_t *like;
    std::vector<int> nidx;   // nuisance_indices, 0-based
    const double *dl;
    long long ld_field, ld_walker;
};

}  // namespace cmamd

struct cmbs {
    cmamd::DevCfg dc{};
    int W = 0, np = 0, n_used = 0;
    std::vector<int> params_used;
    std::string last_error;
    cmamd::DevBuf rot;                  // rotation lists + counters (DevCfg::rot_list / rot_cnt)
    std::vector<int> rot_par;           // per 64-walker range: the counter the next proposing launch appends to
    std::vector<int> rot_lp;            // per 64-walker range: the single fast block's loop index mod n, or -1 (rot_may_pend)
    bool rot_fast_any = false;          // some fast block is wide enough to defer its rotations
    int rot_fast_n = 0;                 // width of the only fast block when it is deferred, else 0
    int stage_R_force = -1;             // debug: rotation rows staged (1) / in HBM (0) / by set_mh_lds (-1)
    cmamd::DevBuf tab_i, tab_d, sd, si, like_terms, cur_terms, ws, hist, hist_terms, mom, itmp_g;
    cmamd::DevBuf nuis_bufs[cmamd::MAXLIKE];
    std::vector<int> h_tab_i;
    std::vector<double> h_tab_d;
    std::vector<cmamd::LikeSlot> likes;
    // host copies of the proposer structure
    std::vector<int> indices, proposer_for_index, blk_start, blk_n, blk_nchanged, used_params_changed_all;
    std::vector<int> blk_changed_off, blk_map_off, blk_R_off, changed;
    int all_n = 0, slow_n = 0, fast_n = 0, nblocks = 0, R_total = 0, map_total = 0;
    size_t mh_lds = 0;
    int hist_cap = 0, hist_count = 0;
    bool started = false;
    // walker groups: contiguous 64-walker-aligned slices [grp0[g], grp0[g+1]) each
    // stepped on its own stream so one group's Metropolis kernel and the other
    // groups' likelihood kernels share the chip (cmbs_set_groups)
    int n_groups = 1;
    std::vector<int> grp0{0};
    hipStream_t streams[cmamd::MAXGROUPS] = {};
    hipEvent_t events[cmamd::MAXGROUPS + 1] = {};
    cmamd::DevBuf ws_g[cmamd::MAXGROUPS];
    // fast dragging (cmbs_step_drag): scratch rows, second likelihood set, end-point theories
    cmamd::DevBuf drag_dd, drag_di, like_terms2;
    cmamd::DevBuf like_ws2[cmamd::MAXLIKE];  // the fused likelihoods' workspaces for the start-point set (drag pairs)
    bool no_drag_pair = false;               // debug: the drag's two evaluation sets one after the other
    bool drag_hbm = false;                   // debug: drag_kernel on the HBM state (cmamd_debug_drag_hbm)
    cmamd::DevBuf nuis_bufs2[cmamd::MAXLIKE];
    struct EndTheory { double *dl = nullptr; long long ld_field = 0, ld_walker = 0; };
    EndTheory end_theory[cmamd::MAXLIKE];
    long long num_drag = 0;
    // the sampler swapped accepted trial theories into the walkers' theory rows
    // (cmbs_step_theory / cmbs_step_drag); after a resume those rows must be
    // recomputed at the restored points (cmbs_refresh_theory) before stepping
    bool theory_moved = false, theory_stale = false;
    // sample collector (collector.hip): per-walker Samples lists over the history ring
    struct Collector {
        cmamd::DevBuf samp, state, flag, wcount, steps;
        int cap = 0;
        bool enabled = false;
    } coll;
    // change mask: flags, per sparse likelihood the compacted walker slots
    // (count, DataParams rows, theory rows when per walker, terms)
    cmamd::DevBuf like_flag, like_cnt;
    cmamd::DevBuf like_outc[cmamd::MAXLIKE], like_nuisc[cmamd::MAXLIKE], like_dlc[cmamd::MAXLIKE];
    std::vector<int> sparse_likes;          // likelihood indices evaluated sparsely
    bool mask_on = false;                   // some likelihood can skip walkers (SetMask at add_likelihood)
    // deferred combines: the likelihoods that may defer (each with a workspace
    // of its own, which must survive until the accepting mh_kernel), and how
    // many the last evaluation left pending in dc.def_*
    std::vector<int> defer_likes;
    cmamd::DevBuf like_ws[cmamd::MAXLIKE];
    int pending_def = 0;
    // fused window pass (theorypass.h): plik_lite and a CMBlikes dataset that
    // read one theory buffer run their window stages as one pass; each then
    // continues from its own workspace (like_ws)
    std::unique_ptr<cmamd::TheoryPass> tpass;
    int tp_like[2] = {-1, -1};               // [0] plik_lite (Delta rows), [1] CMBlikes (partial rows)
    cmamd::WinStage tp_stage[2];
    bool no_corun = false;                   // debug: the fused pass's tails as separate launches
    // the bin co-run's calibration hand-off (mh_bin_kernel)
    cmamd::DevBuf pipe_cal;                  // [2 halves][2 stages][ld] (DevCfg::calbuf)
    unsigned pipe_epoch = 0;                 // proposing bin co-run launches so far (its parity: the half)
    int pipe_ready = 0;                      // set up for this W (0: not yet)
    // fast-step schedule: 3 the unified step launch (default, where it applies;
    // else the bin co-run or the unpipelined steps), 0 unpipelined (debug /
    // A/B: CMAMD_PIPE, cmamd_debug_pipeline)
    int pipe_mode = 3;
    cmamd::DevBuf tail_S[2][2];              // [parity][stage] the pass's raw sums
    cmamd::DevBuf tail_rowcal;               // the chi^2 stage's calibrated partial rows (SmallGaussLaunch::row_cal)
    int tail_ready = 0;                      // W it is set up for (0: not yet, -W: not possible)
    int tail_qf = -1, tail_g = -1;           // the stage (0 / 1) of the quadratic form / of the chi^2
    // unified step launches: one launch per step holds step k's
    // tails, step k + 1's pass and the Metropolis workgroups that accept step k
    // (waiting per tile on the tails: TailWait) and propose step k + 1
    cmamd::DevBuf tail_cnt;                  // [tiles] TailWait::cnt
    size_t tail_cnt_bytes = 0;
    unsigned tail_epoch = 0;
    unsigned tail_epoch_g = 0;               // accepting unified launches with the chi^2 as rows (not folded)
    cmamd::StepTailPlan uni_plan[3];         // rows: propose + pass, tails + pass + accept/propose, tails + accept
    size_t uni_lds = 0;
    int tail_nosignal = 0;                   // debug (cmamd_debug_tail_nosignal)
    bool binned_cache = false;               // cmbs_set_binned_cache: bin once per fast-step call
    int qf_ahead = 1;                        // unified launch: qfs_body_nj in the middle launches too (CMAMD_QF_AHEAD=0: the loop form)
    int fold_late_prio = 0;                  // unified launch: CMAMD_FOLD_LATE_PRIO (A/B)
    int qf_prio = 1;                         // unified launch: the QF waves at priority 2 (CMAMD_QF_PRIO=0 off)
    int fold_tpf = 1;                        // unified launch: CMAMD_FOLD_TPF (A/B, 1 or 2)
    int fold_g = 1;                          // unified launch: the small chi^2 in the Metropolis workgroups
                                             // (CMAMD_FOLD_G=0: as rows of its own, for A/B runs)
    // a pipelined hand-off that gave up (unified launch, bin co-run): the device word, its
    // pinned copy taken at the end of each step call, checked at the next
    int *pipe_status_host = nullptr;         // pinned, mapped (pipe_status_init)
    int *pipe_status_dev = nullptr;          // its device address
    hipEvent_t pipe_ev = nullptr;
    bool pipe_ev_pending = false;
    // bin co-run (a lone plik_lite likelihood, no fused pass): the proposing
    // launch also bins every walker's theory into raw sums (mh_bin_kernel);
    // plik's deferred evaluation continues from them (Like::deferred_from_sums)
    cmamd::DevBuf bin_S;                     // [wpad(W)][Np] raw bin sums (padding zero)
    size_t bin_lds = 0;                      // mh_bin_kernel's LDS
    int tp_why = 0;                          // set-up progress when no pass was built (debug)
    bool lean_off = false;                   // debug: the generic chain where the lean one applies (cmamd_debug_lean)
    ~cmbs() {
        if (pipe_status_host) (void)hipHostFree(pipe_status_host);
        if (pipe_ev) (void)hipEventDestroy(pipe_ev);
        for (auto &st : streams)
            if (st) (void)hipStreamDestroy(st);
        for (auto &e : events)
            if (e) (void)hipEventDestroy(e);
    }
};

namespace cmamd {
void sampler_set_groups(cmbs *s, int n_groups);
// a pipelined hand-off that gave up fails here (wait: for the last step call's copy)
void sampler_check_pipe(cmbs *s, bool wait = false);
void sampler_chain_moments(cmbs *s, int first, int last, const double *gmean, double *out, hipStream_t stream);
void sampler_history_host(cmbs *s, int first, int count, double *out);
void sampler_set_trial_theory(cmbs *s, int like_index, double *dl_end, long long ld_field, long long ld_walker);
void sampler_step_drag(cmbs *s, int n_steps, double dragging_steps, cmbs_theory_fn fn, void *user, hipStream_t stream);
void sampler_step_theory(cmbs *s, int n_steps, cmbs_theory_fn fn, void *user, hipStream_t stream);
void sampler_refresh_theory(cmbs *s, cmbs_theory_fn fn, void *user, hipStream_t stream);
void sampler_collector_enable(cmbs *s, int samp_capacity);
void sampler_collector_add(cmbs *s, const int *steps, int nsteps, int min_update, int check_burn, hipStream_t st);
void sampler_collector_state_host(cmbs *s, int *start, int *count, int *burn, int *thin);
void sampler_collector_thin(cmbs *s, int limit, hipStream_t st);
void sampler_collector_moments(cmbs *s, const double *gmean, double *out, hipStream_t stream);
void sampler_collector_limits(cmbs *s, const int *params, int ncheck, double limfrac, double *out, hipStream_t stream);
size_t sampler_collector_bytes(const cmbs *s);
void sampler_collector_save(cmbs *s, void *buf);
void sampler_collector_load(cmbs *s, const void *buf);
}
