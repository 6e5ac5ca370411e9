/* cosmomc_amd -- MI355X-native fast-parameter likelihood + MCMC step for CosmoMC.
 *
 * C ABI of libcosmomc_amd.so.  Plain pointers and sizes only; every device
 * pointer argument is a HIP device pointer (e.g. torch.Tensor.data_ptr() of a
 * cuda tensor), every stream a hipStream_t (NULL = default stream).
 * Errors are returned as negative codes plus a message (never an abort);
 * the message of the last failing call on a handle is cmbl_last_error().
 *
 * Reference interfaces replaced (SouthPoleTelescope/CosmoMC):
 *   cmbl_open            CMBLikelihood_Add tag dispatch + ReadDatasetFile/ReadIni
 *                        (source/CMB.f90:54-123, source/likelihood.f90:36-66,
 *                         source/CMB.f90:208-303 for PLIK_LITE)
 *   cmbl_info            TDataLikelihood metadata (source/GeneralTypes.f90:105-126):
 *                        nuisance params, cl_lmax(4,4), speed, name
 *   cmbl_derived_info / cmbl_derived_batch
 *                        DataLike%derivedParameters(Theory, DataParams) and its
 *                        '*' names (source/GeneralTypes.f90:504-512, 658-664, 774-776;
 *                        TSmica_planck_derivedParameters source/CMBlikes.f90:1324-1337)
 *   cmbl_loglike_batch   like%LogLike(CMB, Theory, DataParams) for W walkers at once
 *                        (source/CMB.f90:305-329; called from calclike.f90:380)
 *   cmbl_clik_compute_batch  clik_lnlike packing (source/cliklike.f90:129-170) routed
 *                        to the native kernel; returns +lnL like clik_compute
 *   cmbs_*               BlockedProposer (source/propose.f90:53-298) + Metropolis
 *                        (source/MCMC.f90:119-335) + GetLogLike bounds/priors/temperature
 *                        (source/calclike.f90:82-151), batched over W independent chains
 */
#ifndef COSMOMC_AMD_H
#define COSMOMC_AMD_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CMBL_LOGZERO 1e30          /* settings.f90:114 logZero */

enum {
    CMBL_OK = 0,
    CMBL_ERR_ARG = -1,             /* bad argument */
    CMBL_ERR_IO = -2,              /* dataset / data file unreadable */
    CMBL_ERR_FORMAT = -3,          /* dataset content invalid */
    CMBL_ERR_NUMERIC = -4,         /* covariance not positive definite, ... */
    CMBL_ERR_HIP = -5,             /* HIP runtime error */
    CMBL_ERR_UNSUPPORTED = -6      /* dataset type / option not implemented */
};

/* Theory layout: field pair f of Theory%Cls(i,j), i>=j with T=1,E=2,B=3,P=4,
 * f = i*(i-1)/2 + j - 1: TT=0 TE=1 EE=2 BT=3 BE=4 BB=5 PT=6 PE=7 PB=8 PP=9.
 * D_l = l(l+1)C_l/2pi in muK^2 (source/CosmoTheory.f90:25), indexed from l=0:
 *   dl[w*ld_walker + f*ld_field + l]. */
#define CMBL_NFIELDS 10

typedef struct cmbl cmbl_t;

/* tag -> likelihood class as CMBLikelihood_Add (source/CMB.f90:80-97):
 * "PLIK_LITE" native plik_lite (CMB.f90:30-329), "BKPLANCK" CMBlikes with the
 * BICEP/Keck/Planck foregrounds (CMB_BK_Planck.f90), "SPTPOL_TEEE" / "SPTPOL_BB"
 * the SPTpol TE/EE 2017 and BB 2019 likelihoods (CMB_SPTpol_TEEE_2017.f90,
 * CMB_SPTpol_BB_2019.f90; sptpol_blind_r is CMBL_ERR_UNSUPPORTED), "SMICA"
 * CMBlikes with the SMICA TT foreground, nuisance_params and
 * calibration_paramname (TSmica_planck, CMBlikes.f90:1262-1339; binned HL or
 * gaussian), "WMAP" CMBL_ERR_UNSUPPORTED (external library), any other tag a CMBlikes
 * dataset (CMBlikes.f90; like_approx HL or gaussian, binned, or exact,
 * unbinned: ExactChiSq CMBlikes.f90:967-979, up to 4 maps).
 * override_ini: "key = value" lines applied over the dataset file, as
 * cmb_dataset[TAG,key] = value (source/CMB.f90:71-74); may be NULL. */
int  cmbl_open(const char *tag, const char *dataset_path, const char *override_ini,
               cmbl_t **out, char *errbuf, size_t errlen);
void cmbl_close(cmbl_t *h);
const char *cmbl_last_error(const cmbl_t *h);

/* cl_lmax: 16 ints, cl_lmax[(i-1)*4 + (j-1)] = cl_lmax(i,j) (0 = unused).
 * speed: likelihood speed (-1 = slow default of TCMBLikelihood).
 * nuisance_names: space separated names from the calibration/nuisance
 * .paramnames (pointer owned by the handle). */
int  cmbl_info(const cmbl_t *h, int *n_nuis, int *cl_lmax, int *speed,
               const char **name, const char **nuisance_names);

/* Derived parameters a likelihood outputs per sample (the '*' names of its
 * nuisance .paramnames): their count and space-separated names (pointer owned
 * by the handle).  0 for most datasets. */
int  cmbl_derived_info(const cmbl_t *h, int *n_derived, const char **derived_names);

/* The derived parameters at W points (device pointers, asynchronous on
 * `stream`): nuis [W] x n_nuis (stride ld_nuis) as for cmbl_loglike_batch,
 * derived [W] x n_derived (stride ld_derived >= n_derived).  SMICA: the TT
 * foreground D_l at l = 2000 (TSmica_planck_derivedParameters); other
 * datasets: zeros (TDataLikelihood_derivedParameters).  The reference's
 * functions read no theory, so none is passed. */
int  cmbl_derived_batch(cmbl_t *h, int W, const double *nuis, long long ld_nuis,
                        double *derived, long long ld_derived, void *stream);

/* Bytes of device workspace cmbl_loglike_batch needs for W walkers. */
size_t cmbl_workspace_size(const cmbl_t *h, int W);

/* -lnL for W walkers (device pointers, asynchronous on `stream`):
 *   dl    [W] x [10 fields] x [l]  (strides ld_walker, ld_field, 1);
 *         ld_walker = 0 gives every walker the same theory (one slow point)
 *   nuis  [W] x n_nuis (stride ld_nuis)   -- DataParams of each walker
 *   out   [W]
 * workspace: cmbl_workspace_size(h, W) bytes of device memory, or NULL to use
 * the handle's own (then calls on one handle must not overlap). */
int  cmbl_loglike_batch(cmbl_t *h, int W,
                        const double *dl, long long ld_field, long long ld_walker,
                        const double *nuis, long long ld_nuis,
                        double *out, void *workspace, void *stream);

/* Same with HOST arrays: stages through pinned host memory and device buffers
 * the handle keeps between calls (no allocation per call once sized), runs on
 * the handle's own stream and synchronises.  For hosts that keep C_l in CPU
 * memory, e.g. the reference's LogLike called per evaluation with W = 1
 * (INTEGRATION.md).  Reads only the theory the likelihood uses: fields up to
 * the last with cl_lmax > 0, each to its lmax.  One host call at a time per
 * handle (serialised internally). */
int  cmbl_loglike_batch_host(cmbl_t *h, int W,
                             const double *dl, long long ld_field, long long ld_walker,
                             const double *nuis, long long ld_nuis, double *out);

/* clik-compatible entry (source/cliklike.f90:138-166): each walker row of
 * cl_and_pars (stride ld) holds C_l (not D_l) for l=0..lmax of TT, EE, BB,
 * TE, TB, EB (lmax per spectrum from clik_lmax[6], -1 = absent) followed by
 * the nuisance parameters.  Writes +lnL (= -(-lnL)) like clik_compute.
 * Device pointers. */
int  cmbl_clik_compute_batch(cmbl_t *h, int W, const int *clik_lmax,
                             const double *cl_and_pars, long long ld,
                             double *lnlike, void *workspace, void *stream);
/* Device workspace bytes cmbl_clik_compute_batch needs for W walkers
 * (workspace NULL: the handle's own, grown on demand; such calls are serialised
 * on the host and ordered on the device after the previous one, whatever its
 * stream; asynchronous either way). */
size_t cmbl_clik_workspace_size(const cmbl_t *h, int W);

/* Sticky numerical status of a handle, set on device by the likelihood
 * kernels (their -lnL output for the affected walker is NaN):
 *   CMBL_STATUS_HL_NOCONV  an HL eigensolve (CMBLikes_Transform, CMBlikes.f90:
 *                          861-914) did not converge in 40 Jacobi sweeps; the
 *                          reference's LAPACK call would stop the run
 *   CMBL_STATUS_PIPE_WAIT  a sampler's pipelined fast step (cmbs_step) gave up
 *                          waiting for its walkers' trial calibrations, so its
 *                          terms are not to be trusted (a safety net: the wait
 *                          ends by construction)
 * cmbl_status synchronises the device, writes the bits accumulated since the
 * last clear to *flags and clears them when clear != 0.  The host entry
 * (cmbl_loglike_batch_host) checks them itself and returns CMBL_ERR_NUMERIC. */
#define CMBL_STATUS_HL_NOCONV 1
#define CMBL_STATUS_PIPE_WAIT 2
int  cmbl_status(cmbl_t *h, int *flags, int clear);

/* Per-kernel device timing (HIP events around every library launch; off by
 * default).  cmbl_profile_read: accumulated milliseconds and launch count of
 * the kernel named `kernel` (e.g. "plik_quadform_pairs"); synchronises. */
void cmbl_profile_enable(int on);
void cmbl_profile_reset(void);
int  cmbl_profile_read(const char *kernel, double *total_ms, long long *count);

/* ------------------------------------------------------------------ */
/* Batched Metropolis sampler (W independent chains, one per walker).  */

typedef struct cmbs cmbs_t;

typedef struct {
    int n_walkers;
    int num_params;            /* length of P (all parameters, used or fixed) */
    int n_used;                /* number of varying parameters */
    const int *params_used;    /* n_used, 1-based indices into P (settings.f90:97) */
    int n_blocks;              /* BaseParams%param_blocks (slow -> fast) */
    const int *block_n;        /* n_blocks sizes */
    const int *block_params;   /* concatenated, 1-based indices into params_used */
    int slow_block_max;        /* blocks 1..slow_block_max are slow (propose.f90:151) */
    int oversample_fast;
    double propose_scale;      /* MCMC.f90:38 default 2.4 */
    double temperature;        /* calclike.f90 Temperature */
    const double *pmin, *pmax; /* num_params hard bounds */
    const double *prior_mean, *prior_std; /* num_params Gaussian priors, std 0 = none */
    int seed_ij, seed_kl;      /* RANMAR seeds of walker 0; walker w uses
                                  cmbs_walker_seed() (documented in DESIGN.md) */
    int first_walker;          /* global index of walker 0 (for sharding) */
    /* GetLogPriors (calclike.f90:111-134): a Gaussian prior on parameter i counts
     * when i is varying (in params_used) or include_fixed_parameter_priors is set
     * (BaseParameters.f90:170-181); linear-combination priors
     * ((dot(weights, P) - mean)/std)^2 over all num_params (:184-201), std 0 = none */
    int include_fixed_parameter_priors;
    int n_lincomb;
    const double *lincomb_weights;              /* n_lincomb x num_params, row-major */
    const double *lincomb_mean, *lincomb_std;   /* n_lincomb */
} cmbs_config_t;

/* walker w's RANMAR seeds (ij in 0..31328, kl in 0..30081) */
void cmbs_walker_seed(int seed_ij, int seed_kl, int walker, int *ij, int *kl);

int  cmbs_create(const cmbs_config_t *cfg, cmbs_t **out, char *errbuf, size_t errlen);
void cmbs_destroy(cmbs_t *s);
const char *cmbs_last_error(const cmbs_t *s);

/* proposal covariance of the used parameters, n_used x n_used row-major host
 * array (BlockedProposer_SetCovariance, propose.f90:210-244) */
int  cmbs_set_covariance(cmbs_t *s, const double *cov);

/* test_likelihood term (calclike.f90:180-199): -lnL += (P-c)^T C^-1 (P-c)/2
 * over params_used; cov is n_used x n_used (inverted here), center num_params. */
int  cmbs_set_test_gaussian(cmbs_t *s, const double *cov, const double *center);

/* Add a CMB likelihood evaluated on cached per-walker theory:
 * DataParams = P(nuisance_indices) (GeneralTypes.f90:642-646: the indices
 * AddNuisanceParameters assigns, :618-669, in any order and shared between
 * likelihoods, e.g. calPlanck for plik_lite and lensing), nuisance_indices
 * 1-based, n_nuis of them (cmbl_info).  dl is a device array laid out as for
 * cmbl_loglike_batch for this sampler's walkers; it must stay alive while the
 * sampler is used. */
int  cmbs_add_likelihood(cmbs_t *s, cmbl_t *like, const int *nuisance_indices,
                         const double *dl, long long ld_field, long long ld_walker);

/* Initial points (host, W x num_params) -> evaluates the starting -lnL. */
int  cmbs_set_start(cmbs_t *s, const double *P0, void *stream);

/* n_steps Metropolis steps for every walker.  fast_only != 0:
 * FastParameterSample (MCMC.f90:309-335, GetProposalFast) every step;
 * otherwise TMetropolisSampler_GetNewSample (MCMC.f90:269-307, GetProposal).
 * Asynchronous on stream.  The pipelined fast-step schedules hand data from
 * one workgroup to another inside a launch with bounded waits; a wait that
 * gives up marks the call's steps invalid, and the next cmbs_step or state /
 * history readback returns CMBL_ERR_NUMERIC ("... gave up waiting ..."). */
int  cmbs_step(cmbs_t *s, int n_steps, int fast_only, void *stream);

/* Fast dragging, TFastDraggingSampler_GetNewSample (MCMC.f90:338-452;
 * sampling_method = fast_dragging): n_steps GetNewSample calls for every
 * walker; every oversample_fast-th call drags the fast parameters (Neal) along
 * a slow proposal over interp_steps = max(2, nint(dragging_steps * num_fast) + 1)
 * interpolation steps (dragging_steps 3 by default, settings.f90:82), the
 * others are FastParameterSample.  Each drag needs the likelihoods at the
 * proposed slow point: `theory_fn` is called once per drag (synchronously,
 * after the slow proposal) with the device trial rows P_end [num_params][ld]
 * (walker-minor) and must fill every likelihood's end-theory buffer
 * registered with cmbs_set_trial_theory; it returns 0 on success.  Walkers
 * whose drag is accepted get their end theory copied into their theory rows
 * (the dl buffer passed to cmbs_add_likelihood).  With no likelihoods (the
 * analytic test target) theory_fn may be NULL.  Walkers whose CurLike is
 * logZero skip the drag (the reference makes a full Metropolis step there). */
typedef int (*cmbs_theory_fn)(void *user, int W, const double *P_end, long long ld, void *stream);
/* Trial-point theory buffer of likelihood `like_index` (same layout as its
 * theory rows), filled by the theory function for dragging end points and
 * for cmbs_step_theory trial points. */
int  cmbs_set_trial_theory(cmbs_t *s, int like_index, double *dl_end, long long ld_field, long long ld_walker);
int  cmbs_step_drag(cmbs_t *s, int n_steps, double dragging_steps, cmbs_theory_fn theory_fn, void *user,
                    void *stream);
/* Full TMetropolisSampler_GetNewSample steps (MCMC.f90:269-307; GetProposal
 * slow and fast) when data likelihoods need the theory at the trial point
 * (the reference recomputes it with CAMB, CalcLike_Cosmology.f90:59-94):
 * theory_fn fills the trial-theory buffers from the trial rows every step and
 * accepted walkers take the trial theory.  cmbs_step(fast_only = 0) refuses
 * slow proposals when data likelihoods are registered. */
int  cmbs_step_theory(cmbs_t *s, int n_steps, cmbs_theory_fn theory_fn, void *user, void *stream);

/* After cmbs_load_state of an image whose walkers moved their slow parameters
 * (cmbs_step_theory / cmbs_step_drag ran before the checkpoint), the walker
 * theory rows given to cmbs_add_likelihood hold whatever the new process put
 * there: every cmbs_step* call fails until this refreshes them.  theory_fn is
 * called once with the current points P [num_params][ld] and fills every
 * trial-theory buffer (cmbs_set_trial_theory), which is then copied into the
 * walkers' theory rows.  The reference likewise recomputes the theory at the
 * restart point (GeneralSetup.f90:123-131).  CurLike and the per-likelihood
 * terms stay as saved (not re-evaluated): theory_fn must reproduce the theory
 * the run had at those points. */
int  cmbs_refresh_theory(cmbs_t *s, cmbs_theory_fn theory_fn, void *user, void *stream);

/* Execution tuning (no reference counterpart; results are unchanged): split the
 * walkers into n_groups 64-aligned slices, each stepped on an internal stream
 * forked from / joined to the caller's, so the Metropolis kernel of one slice
 * overlaps the likelihood kernels of the others.  Default 1. */
int  cmbs_set_groups(cmbs_t *s, int n_groups);

/* Binned-theory cache (SURVEY 8(d)'s labelled variant, no reference
 * counterpart): inside one cmbs_step call of fast-only steps the theory is
 * fixed, and the window/bin sums of the theory are calibration-independent,
 * so with on != 0 the unified fast step bins each walker's theory once per
 * call and every step reuses those raw sums (the quadratic form, the small
 * chi^2 and the Metropolis chain still run every step, and the calibration is
 * applied to the sums as before, so the results are the same bits).  Only the
 * unified schedule (plik_lite + a small gaussian CMBlikes likelihood) uses it;
 * other runs ignore it.  Default 0: every step re-bins the theory, as the
 * reference's LogLike does. */
int  cmbs_set_binned_cache(cmbs_t *s, int on);

/* Optional history capture for convergence statistics: every step appends
 * each walker's current used-parameter vector and CurLike to a device ring of
 * `capacity` steps (SampleCollector AddNewPoint, SampleCollector.f90:324-456). */
int  cmbs_enable_history(cmbs_t *s, int capacity);
/* Per-walker statistics over history rows [first, last] (inclusive; row k is
 * the k-th step recorded since cmbs_enable_history, the ring keeps the last
 * `capacity`): means[W][n_used], covs[W][n_used][n_used], device ptrs
 * (SampleCollector.f90:235-246 "second half" window is first = count/2). */
int  cmbs_history_stats(cmbs_t *s, int first, int last, double *means, double *covs, void *stream);
int  cmbs_history_count(const cmbs_t *s);
/* Synchronising copy of history rows [first, first+count) (step indices as
 * cmbs_history_stats; the ring keeps the last `capacity`) to HOST memory: out[count][n_used + 1][W], per step the used parameters
 * then CurLike of every walker (the chain-file writer's input,
 * IO_OutputChainRow IO.f90:85-93). */
int  cmbs_history_host(cmbs_t *s, int first, int count, double *out);
/* This GPU's partial sums for the convergence / proposal-learning exchange
 * (TMpiChainCollector_UpdateCovAndCheckConverge, SampleCollector.f90:212-322):
 * each walker is one chain whose samples are history rows [first, last].
 * Device out:
 *   gmean == NULL: [sum count, sum count*mean (n), sum count*cov (n*n),
 *                   sum cov (n*n), number of chains]      (2 + n + 2n^2)
 *   gmean != NULL: sum count*(mean-gmean)(mean-gmean)^T    (n^2)
 * where n = n_used.  Summed over GPUs these give the reference's pooled
 * mean, MPICovMat, mean-of-covariances and covariance-of-means. */
int  cmbs_chain_moments(cmbs_t *s, int first, int last, const double *gmean, double *out, void *stream);

/* Sample collector (TMpiChainCollector_AddNewPoint, SampleCollector.f90:324-460):
 * every walker's Samples list -- the thinned points the convergence test
 * windows over -- kept on device as a ring of history step numbers (the points
 * stay in the history ring).  cmbs_collector_enable after cmbs_enable_history;
 * sample_capacity bounds each walker's list (Samples%Thin keeps it below
 * the reference's 500000).  Part of the cmbs_save_state image once enabled. */
int  cmbs_collector_enable(cmbs_t *s, int sample_capacity);
/* AddNewPoint for history steps steps[0..n_steps) (increasing; host array)
 * of every walker: sample_num++, keep every MPI_thin_fac-th, Samples%Add (points
 * at logZero are skipped, MCMC.f90:146); with check_burn, the burn-in test
 * (a used parameter changed > 51 times between consecutive samples once
 * Count > 51, :352-377) and on burn DeleteRange to the last min_sample_update
 * samples (:391-397).  Synchronises; fails if a list outgrows its capacity. */
int  cmbs_collector_add(cmbs_t *s, const int *steps, int n_steps, int min_sample_update, int check_burn,
                        void *stream);
/* HOST copies of every walker's list start/count, Burn_done and MPI_thin_fac (any may be NULL). */
int  cmbs_collector_state_host(cmbs_t *s, int *start, int *count, int *burn_done, int *thin_fac);
/* Samples%Thin(2) and MPI_thin_fac * 2 for every walker whose Count > limit (:300-304). */
int  cmbs_collector_thin(cmbs_t *s, int limit, void *stream);
/* As cmbs_chain_moments, each walker over its own window: items Count/2 .. Count
 * of its list, Count - Count/2 + 1 samples (:233-246), its weight in the sums. */
int  cmbs_collector_moments(cmbs_t *s, const double *gmean, double *out, void *stream);
/* CheckLimitsConverge's per-chain limits (:477-544): ConfidVal (samples.f90:70-110)
 * of used parameters params[0..n_check) (0-based) over each walker's window at
 * limfrac (MPI_Limit_Converge): out[W][n_check][2] = (lower, upper), device
 * pointer; synchronises. */
int  cmbs_collector_limits(cmbs_t *s, const int *params, int n_check, double limfrac, double *out, void *stream);

/* Device pointers of the walker state (valid until destroy), walker-minor:
 * P [num_params][W], cur_like [W], mult [W] (double), num_accept [W] (int). */
int  cmbs_state(cmbs_t *s, double **P, double **cur_like, double **mult, int **num_accept);

/* Synchronising copy of the walker state to HOST arrays (any may be NULL):
 * P [W][num_params], cur_like [W], mult [W], num_accept [W]. */
int  cmbs_get_state_host(cmbs_t *s, double *P, double *cur_like, double *mult, int *num_accept);

/* Checkpoint / resume (replaces TMpiChainCollector_SaveState / ReadState,
 * SampleCollector.f90:139-202, and TChainSampler_SaveState / LoadState,
 * MCMC.f90:199-218).  The image is every walker's complete chain state
 * (point, CurLike, multiplicity, accept count, RANMAR state, proposer
 * cycle/rotation state), so a resumed chain continues exactly where it
 * stopped; the reference restarts from the last chain row with a new random
 * sequence instead.  The proposal covariance is not in the image: restore it
 * with cmbs_set_covariance first.  Loading checks the sampler shape and marks
 * the sampler started (no cmbs_set_start needed). */
size_t cmbs_state_bytes(const cmbs_t *s);
int  cmbs_save_state(cmbs_t *s, void *host_buf, size_t bytes);
int  cmbs_load_state(cmbs_t *s, const void *host_buf, size_t bytes);

/* Each likelihood's -lnL at the recorded points, history rows [first,
 * first + count), to HOST memory: out[count][n_likelihoods][W] in
 * cmbs_add_likelihood order (TCalculationAtParamPoint%Likelihoods: the
 * chi2_<tag> = 2 x term derived columns of a chain row, GeneralTypes.f90:767-776). */
int  cmbs_history_terms_host(cmbs_t *s, int first, int count, double *out);

/* Put history rows [first, first + count) back (HOST arrays laid out as
 * cmbs_history_host / cmbs_history_terms_host write them, terms may be NULL;
 * count <= capacity) and continue the ring at first + count: the samples the
 * convergence exchange windows over survive a resume (Samples%LoadState,
 * SampleCollector.f90:167). */
int  cmbs_history_restore(cmbs_t *s, int first, int count, const double *rows, const double *terms);

#ifdef __cplusplus
}
#endif
#endif
