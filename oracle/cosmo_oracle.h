/* ORACLE TEST INFRASTRUCTURE -- CPU restatement of the reference's fast-path
 * arithmetic.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load liboracle.so, and only as the checker / CPU
 * baseline.  The product library (cosmomc_amd/lib) never links it.
 *
 * Every routine cites the reference file:line it restates.  The restatement
 * itself is pinned against the compiled reference (oracle/_ref, built by
 * oracle/Makefile from /root/reference/source) through the JSON fixtures in tests/golden/.
 */
#ifndef COSMO_ORACLE_H
#define COSMO_ORACLE_H
#ifdef __cplusplus
extern "C" {
#endif

#define ORC_LOGZERO 1e30                 /* settings.f90:114 */

/* ---------------- RandUtils.f90 ---------------- */
typedef struct {
    double u[97];
    double c, cd, cm;
    int i97, j97;
    int iset;                            /* Gaussian1 cache, RandUtils.f90:159-177 */
    double gset;
} orc_rng_t;

void   orc_rmarin(orc_rng_t *r, int ij, int kl);            /* RandUtils.f90:286-348 */
double orc_ranmar(orc_rng_t *r);                             /* RandUtils.f90:350-374 */
double orc_gaussian1(orc_rng_t *r);                          /* RandUtils.f90:156-178 */
float  orc_randexp1(orc_rng_t *r);                           /* RandUtils.f90:189-233 */
void   orc_rand_indices(orc_rng_t *r, int *indices, int nmax, int n);   /* :93-108, 1-based */
void   orc_rand_rotation(orc_rng_t *r, double *R, int n);   /* :133-153, R row-major R[j*n+i]=R(j+1,i+1) */

/* ---------------- Matrix_utils_new.f90 ---------------- */
int    orc_cholesky_lower(double *A, int n);                 /* dpotrf 'L' (Matrix_Cholesky :1339-1369) */
int    orc_matrix_inverse(double *A, int n);                 /* Matrix_Inverse :1515-1569 (dpotrf+dpotri) */
double orc_quadform(const double *M, const double *v, int n);/* Matrix_QuadForm :2033-2047 (DSYMV 'U'+DDOT) */

/* ---------------- CMB.f90 TPlikLiteLikelihood ---------------- */
typedef struct orc_plik orc_plik_t;
/* dataset selection as TPlikLiteLikelihood_ReadIni (CMB.f90:208-303):
 * use_mask bit0 TT, bit1 TE, bit2 EE; range_min/range_max = bins_for_L_range
 * (range_min < 0 => unset).  blmin/blmax are the on-disk 0-based offsets. */
orc_plik_t *orc_plik_create(int plmin, int nweights, const double *weights_file,
                            const long *blmin_off, const long *blmax_off, int maxbin,
                            const int nbincl[3], int use_mask, int range_min, int range_max,
                            const double *X_full, const double *cov_full, int nbins_total);
int    orc_plik_nused(const orc_plik_t *p);
/* CMB.f90:305-329. dl: field-pair blocks (TT, TE, EE at fields 0,1,2), each
 * indexed by l from 0, ld_field doubles apart. */
double orc_plik_loglike(const orc_plik_t *p, const double *dl, long ld_field, double cal);
void   orc_plik_free(orc_plik_t *p);

/* ---------------- propose.f90 BlockedProposer ---------------- */
typedef struct orc_proposer orc_proposer_t;
/* blocks: nblocks blocks, block b has block_n[b] parameter indices (1-based
 * "used" numbering, like BaseParams%param_blocks) in block_params (concatenated);
 * slow_block_max as in Init (propose.f90:151-208). params_used maps used
 * index -> full parameter index (1-based), n_used entries. */
orc_proposer_t *orc_proposer_create(int nblocks, const int *block_n, const int *block_params,
                                    int slow_block_max, int oversample_fast, double propose_scale,
                                    int n_used, const int *params_used);
void orc_proposer_set_covariance(orc_proposer_t *p, const double *cov); /* :210-244, n_used^2 */
void orc_proposer_get_proposal(orc_proposer_t *p, orc_rng_t *r, double *P);        /* :257-273 */
void orc_proposer_get_proposal_slow(orc_proposer_t *p, orc_rng_t *r, double *P);   /* :275-281 */
void orc_proposer_get_proposal_fast(orc_proposer_t *p, orc_rng_t *r, double *P);   /* :283-289 */
void orc_proposer_get_proposal_fast_delta(orc_proposer_t *p, orc_rng_t *r, double *P, int num_params); /* :291-298 */
int  orc_proposer_slow_n(const orc_proposer_t *p);
int  orc_proposer_fast_n(const orc_proposer_t *p);
void orc_proposer_free(orc_proposer_t *p);

/* ---------------- calclike.f90 + MCMC.f90 ---------------- */
typedef struct {
    int num_params;
    const double *pmin, *pmax;          /* GetLogLikeBounds calclike.f90:97-109 */
    const double *prior_mean, *prior_std; /* GetLogPriors :111-134 (std==0 -> none) */
    double temperature;                 /* AddLikeTemp :82-94 */
    /* test_likelihood (calclike.f90:180-199): X = P(params_used)-center */
    int test_like, n_used;
    const int *params_used;             /* 1-based */
    const double *test_covinv;          /* n_used^2 (already inverted) */
    const double *center;               /* num_params */
    /* native plik_lite on cached theory: DataParams(1)=P(plik_nuis_index) */
    const orc_plik_t *plik;
    int plik_nuis_index;                /* 1-based */
    const double *plik_dl;
    long plik_ld_field;
    /* slow-theory test model: theory = P(plik_scale_index) x plik_dl (0: off),
     * standing in for CAMB's recomputation at the trial point */
    int plik_scale_index;               /* 1-based */
    /* GetLogPriors gate (calclike.f90:119): a Gaussian prior on parameter i
     * counts when varying[i] (NULL: every parameter varies) or
     * include_fixed_parameter_priors; linear-combination priors :125-131 */
    int include_fixed_parameter_priors;
    const int *varying;                 /* num_params flags or NULL */
    int n_lincomb;
    const double *lincomb_weights;      /* n_lincomb x num_params */
    const double *lincomb_mean, *lincomb_std;
    /* further data likelihoods after plik_lite, in DataLikelihoods order
     * (LogLikeWithTheorySet :374-387 sums Params%Likelihoods in list order):
     * -lnL of one more likelihood at P, logZero rejects (NULL: none).  The
     * tests pass a CMBlikes restatement (oracle/cmblikes_oracle.py) here. */
    double (*extra_like)(void *user, const double *P);
    void *extra_user;
} orc_target_t;

double orc_target_loglike(const orc_target_t *t, const double *P); /* GetLogLike :136-151 */
int    orc_metropolis_accept(orc_rng_t *r, double like, double cur_like); /* MCMC.f90:119-131 */

/* One TMetropolisSampler_GetNewSample (MCMC.f90:269-307) or, with fast_only,
 * one FastParameterSample (MCMC.f90:309-335).  Updates P/cur_like in place,
 * returns 1 if accepted.  trial_like_out receives the evaluated -lnL. */
int orc_mh_step(orc_proposer_t *prop, orc_rng_t *r, const orc_target_t *t,
                double *P, double *cur_like, int fast_only, double *trial_like_out);

/* TFastDraggingSampler_GetNewSample (MCMC.f90:338-452): num_drag / mult are
 * the sampler's counters (in/out); dragging_steps as settings.f90:82 (3).
 * Every oversample_fast-th call drags (slow proposal + interp_steps-1
 * fast-delta steps on the start/end interpolated likelihood), the others
 * are FastParameterSample.  Returns 1 if the move was accepted. */
typedef struct { int num_drag; double mult; double dragging_steps; int oversample_fast; } orc_drag_state_t;
int orc_drag_step(orc_proposer_t *prop, orc_rng_t *r, const orc_target_t *t, orc_drag_state_t *st,
                  double *P, double *cur_like);

/* ---------------- samples.f90 GelmanRubinEvalues ---------------- */
/* samples.f90:41-67 restated: cov = mean of per-chain covs, meanscov = cov of
 * the chain means (normalisations as SampleCollector.f90:257-274 pass them);
 * returns max eigenvalue of L^-1 meanscov L^-T with L = chol(cov) (normalised
 * by sqrt(diag cov)). */
double orc_gelman_rubin(const double *cov, const double *meanscov, int n);

#ifdef __cplusplus
}
#endif
#endif
