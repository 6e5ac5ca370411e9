/* ORACLE TEST INFRASTRUCTURE -- CPU restatement of the reference's fast-path
 * arithmetic (see cosmo_oracle.h).  Plain C11, no BLAS: the BLAS/LAPACK
 * calls of the reference are restated with the reference-BLAS loop orders.
 * Compile with -ffp-contract=off (oracle/Makefile) so float RANDEXP1 and the
 * double loops round exactly as written.
 */
#include "cosmo_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* settings.f90:26-27: pi, twopi = 2*pi (double precision) */
#define ORC_TWOPI (2.0 * 3.14159265358979323846264338328)

/* ======================= RandUtils.f90 ======================= */

void orc_rmarin(orc_rng_t *r, int ij, int kl)
{   /* RandUtils.f90:286-348 (Marsaglia-Zaman-James RANMAR init) */
    int i = (ij / 177) % 177 + 2;
    int j = ij % 177 + 2;
    int k = (kl / 169) % 178 + 1;
    int l = kl % 169;
    for (int ii = 0; ii < 97; ii++) {
        double s = 0.0, t = 0.5;
        for (int jj = 0; jj < 24; jj++) {
            int m = (((i * j) % 179) * k) % 179;
            i = j; j = k; k = m;
            l = (53 * l + 1) % 169;
            if ((l * m) % 64 >= 32) s += t;
            t *= 0.5;
        }
        r->u[ii] = s;
    }
    /* 362436.0/16777216.0 etc. are single-precision literals in the
     * reference; both quotients are exact in binary. */
    r->c = 362436.0 / 16777216.0;
    r->cd = 7654321.0 / 16777216.0;
    r->cm = 16777213.0 / 16777216.0;
    r->i97 = 97;
    r->j97 = 33;
    r->iset = 0;
    r->gset = 0.0;
}

double orc_ranmar(orc_rng_t *r)
{   /* RandUtils.f90:350-374 */
    double uni = r->u[r->i97 - 1] - r->u[r->j97 - 1];
    if (uni < 0.0) uni += 1.0;
    r->u[r->i97 - 1] = uni;
    if (--r->i97 == 0) r->i97 = 97;
    if (--r->j97 == 0) r->j97 = 97;
    r->c -= r->cd;
    if (r->c < 0.0) r->c += r->cm;
    uni -= r->c;
    if (uni < 0.0) uni += 1.0;
    return uni;
}

double orc_gaussian1(orc_rng_t *r)
{   /* RandUtils.f90:156-178, polar Box-Muller with the saved second deviate */
    if (r->iset == 0) {
        double v1, v2, rr = 2.0;
        do {
            v1 = 2.0 * orc_ranmar(r) - 1.0;
            v2 = 2.0 * orc_ranmar(r) - 1.0;
            rr = v1 * v1 + v2 * v2;
        } while (rr >= 1.0);
        double fac = sqrt(-2.0 * log(rr) / rr);
        r->gset = v1 * fac;
        r->iset = 1;
        return v2 * fac;
    }
    r->iset = 0;
    return r->gset;
}

float orc_randexp1(orc_rng_t *r)
{   /* RandUtils.f90:189-233, Ahrens-Dieter EA in REAL(4) */
    const float alog2 = 0.6931471805599453f;
    const float a = 5.7133631526454228f;
    const float b = 3.4142135623730950f;
    const float c = -1.6734053240284925f;
    const float p = 0.9802581434685472f;
    const float aa = 5.6005707569738080f;
    const float bb = 3.3468106480569850f;
    const float hh = 0.0026106723602095f;
    const float dd = 0.0857864376269050f;
    float u = (float)orc_ranmar(r);
    while (u <= 0.0f) u = (float)orc_ranmar(r);
    float g = c;
    u = u + u;
    while (u < 1.0f) {
        g = g + alog2;
        u = u + u;
    }
    u = u - 1.0f;
    if (u <= p) return g + aa / (bb - u);
    for (;;) {
        u = (float)orc_ranmar(r);
        float y = a / (b - u);
        float up = (float)orc_ranmar(r);
        float bu = b - u;
        if ((up * hh + dd) * (bu * bu) <= expf(-(y + c))) return g + y;
    }
}

void orc_rand_indices(orc_rng_t *r, int *indices, int nmax, int n)
{   /* RandUtils.f90:93-108; values 1-based like the reference */
    int *tmp = (int *)malloc(sizeof(int) * (size_t)nmax);
    for (int i = 0; i < nmax; i++) tmp[i] = i + 1;
    for (int i = 1; i <= n; i++) {
        int ix = (int)(orc_ranmar(r) * (nmax + 1 - i)) + 1;
        indices[i - 1] = tmp[ix - 1];
        tmp[ix - 1] = tmp[nmax + 1 - i - 1];
    }
    free(tmp);
}

void orc_rand_rotation(orc_rng_t *r, double *R, int n)
{   /* RandUtils.f90:133-153: rows are Gram-Schmidt'ed Gaussian vectors */
    double *vec = (double *)malloc(sizeof(double) * (size_t)n);
    for (int j = 0; j < n; j++) {
        double norm;
        for (;;) {
            for (int i = 0; i < n; i++) vec[i] = orc_gaussian1(r);
            for (int i = 0; i < j; i++) {
                double s = 0.0;
                for (int k = 0; k < n; k++) s += vec[k] * R[i * n + k];
                for (int k = 0; k < n; k++) vec[k] = vec[k] - s * R[i * n + k];
            }
            norm = 0.0;
            for (int k = 0; k < n; k++) norm += vec[k] * vec[k];
            if (norm > 1e-3) break;
        }
        double sn = sqrt(norm);
        for (int k = 0; k < n; k++) R[j * n + k] = vec[k] / sn;
    }
    free(vec);
}

/* ======================= Matrix_utils_new.f90 ======================= */

int orc_cholesky_lower(double *A, int n)
{   /* dpotrf('L') as called by Matrix_Cholesky (Matrix_utils_new.f90:1339-1369);
     * A row-major symmetric; on exit lower triangle = L, upper zeroed. */
    for (int j = 0; j < n; j++) {
        double d = A[j * n + j];
        for (int k = 0; k < j; k++) d -= A[j * n + k] * A[j * n + k];
        if (!(d > 0.0)) return j + 1;
        d = sqrt(d);
        A[j * n + j] = d;
        for (int i = j + 1; i < n; i++) {
            double s = A[i * n + j];
            for (int k = 0; k < j; k++) s -= A[i * n + k] * A[j * n + k];
            A[i * n + j] = s / d;
        }
    }
    for (int i = 0; i < n; i++)
        for (int j = i + 1; j < n; j++) A[i * n + j] = 0.0;
    return 0;
}

static void lower_inverse(double *L, int n)
{   /* dtrtri('L','N'): in-place inverse of a lower-triangular matrix */
    for (int j = 0; j < n; j++) {
        L[j * n + j] = 1.0 / L[j * n + j];
        for (int i = j + 1; i < n; i++) {
            double s = 0.0;
            for (int k = j; k < i; k++) s += L[i * n + k] * L[k * n + j];
            L[i * n + j] = -s / L[i * n + i];
        }
    }
}

int orc_matrix_inverse(double *A, int n)
{   /* Matrix_Inverse -> Matrix_Inverse_Chol (Matrix_utils_new.f90:1478-1569):
     * A = L L^T, A^-1 = L^-T L^-1, symmetrised. */
    for (int i = 0; i < n; i++)
        if (fabs(A[i * n + i]) < 1e-30) return -1;
    int info = orc_cholesky_lower(A, n);
    if (info) return info;
    lower_inverse(A, n);
    double *T = (double *)malloc(sizeof(double) * (size_t)n * n);
    for (int i = 0; i < n; i++)
        for (int j = 0; j <= i; j++) {
            double s = 0.0;
            for (int k = i; k < n; k++) s += A[k * n + i] * A[k * n + j];
            T[i * n + j] = s;
            T[j * n + i] = s;
        }
    memcpy(A, T, sizeof(double) * (size_t)n * n);
    free(T);
    return 0;
}

double orc_quadform(const double *M, const double *v, int n)
{   /* Matrix_QuadForm (Matrix_utils_new.f90:2033-2047): out = DSYMV('U', M, v)
     * (reference-BLAS loop over the upper triangle), then DDOT(v, out). */
    double *y = (double *)calloc((size_t)n, sizeof(double));
    for (int j = 0; j < n; j++) {
        double temp1 = v[j], temp2 = 0.0;
        for (int i = 0; i < j; i++) {
            double a = M[(size_t)i * n + j];   /* A(i,j), upper */
            y[i] += temp1 * a;
            temp2 += a * v[i];
        }
        y[j] += temp1 * M[(size_t)j * n + j] + temp2;
    }
    double s = 0.0;
    for (int i = 0; i < n; i++) s += v[i] * y[i];
    free(y);
    return s;
}

/* ======================= CMB.f90 plik_lite ======================= */

struct orc_plik {
    int plmin, nweights, nused;
    int used[3];
    int nb_used[3];
    int *bins[3];          /* 1-based bin numbers per spectrum */
    int *blmin, *blmax;    /* absolute l */
    double *weights;       /* index l - plmin, pre-multiplied by 2pi/(l(l+1)) */
    double *X;             /* nused */
    double *invcov;        /* nused^2 */
};

orc_plik_t *orc_plik_create(int plmin, int nweights, const double *weights_file,
                            const long *blmin_off, const long *blmax_off, int maxbin,
                            const int nbincl[3], int use_mask, int range_min, int range_max,
                            const double *X_full, const double *cov_full, int nbins_total)
{   /* TPlikLiteLikelihood_ReadIni, CMB.f90:208-303 */
    orc_plik_t *p = (orc_plik_t *)calloc(1, sizeof(orc_plik_t));
    p->plmin = plmin;
    p->nweights = nweights;
    p->blmin = (int *)malloc(sizeof(int) * (size_t)maxbin);
    p->blmax = (int *)malloc(sizeof(int) * (size_t)maxbin);
    for (int i = 0; i < maxbin; i++) {
        p->blmin[i] = (int)blmin_off[i] + plmin;     /* :225 */
        p->blmax[i] = (int)blmax_off[i] + plmin;     /* :227 */
    }
    p->weights = (double *)malloc(sizeof(double) * (size_t)nweights);
    for (int i = 0; i < nweights; i++) {              /* :230-233 */
        double ls = (double)(plmin + i);
        p->weights[i] = weights_file[i] * ORC_TWOPI / ls / (ls + 1.0);
    }
    int mb = nbincl[0];
    for (int i = 1; i < 3; i++) if (nbincl[i] > mb) mb = nbincl[i];
    int *usebins = NULL, nusebins = 0;
    if (range_min >= 0) {                             /* :250-263 */
        usebins = (int *)malloc(sizeof(int) * (size_t)mb);
        for (int i = 1; i <= mb; i++) {
            double centre = (p->blmin[i - 1] + p->blmax[i - 1]) / 2.0;
            if (range_min <= centre && centre <= range_max) usebins[nusebins++] = i;
        }
    }
    p->nused = 0;
    for (int s = 0; s < 3; s++) {                     /* :268-279 */
        p->used[s] = (use_mask >> s) & 1;
        p->bins[s] = NULL;
        p->nb_used[s] = 0;
        if (!p->used[s]) continue;
        p->bins[s] = (int *)malloc(sizeof(int) * (size_t)nbincl[s]);
        if (usebins) {
            for (int k = 0; k < nusebins; k++)
                if (usebins[k] <= nbincl[s]) p->bins[s][p->nb_used[s]++] = usebins[k];
        } else {
            for (int k = 1; k <= nbincl[s]; k++) p->bins[s][p->nb_used[s]++] = k;
        }
        p->nused += p->nb_used[s];
    }
    int *used_idx = (int *)malloc(sizeof(int) * (size_t)(p->nused > 0 ? p->nused : 1));
    int off = 0, o = 0;
    for (int s = 0; s < 3; s++) {                     /* :285-297 */
        if (p->used[s])
            for (int k = 0; k < p->nb_used[s]; k++) used_idx[o++] = p->bins[s][k] + off - 1;
        off += nbincl[s];
    }
    p->X = (double *)malloc(sizeof(double) * (size_t)p->nused);
    p->invcov = (double *)malloc(sizeof(double) * (size_t)p->nused * p->nused);
    for (int i = 0; i < p->nused; i++) {              /* :298-299 */
        p->X[i] = X_full[used_idx[i]];
        for (int j = 0; j < p->nused; j++)
            p->invcov[(size_t)i * p->nused + j] = cov_full[(size_t)used_idx[i] * nbins_total + used_idx[j]];
    }
    free(used_idx);
    free(usebins);
    if (orc_matrix_inverse(p->invcov, p->nused) != 0) {   /* :300 */
        orc_plik_free(p);
        return NULL;
    }
    return p;
}

int orc_plik_nused(const orc_plik_t *p) { return p->nused; }

double orc_plik_loglike(const orc_plik_t *p, const double *dl, long ld_field, double cal)
{   /* TPlikLiteLikelihood_LogLike, CMB.f90:305-329 */
    double *cl = (double *)malloc(sizeof(double) * (size_t)p->nused);
    int ix = 0;
    for (int s = 0; s < 3; s++) {
        if (!p->used[s]) continue;
        const double *D = dl + (long)s * ld_field;   /* pairs (1,1) (2,1) (2,2) = fields 0,1,2 */
        for (int k = 0; k < p->nb_used[s]; k++) {
            int b = p->bins[s][k] - 1;
            double acc = 0.0;
            for (int l = p->blmin[b]; l <= p->blmax[b]; l++) acc += D[l] * p->weights[l - p->plmin];
            cl[ix++] = acc;
        }
    }
    double c2 = cal * cal;
    for (int i = 0; i < p->nused; i++) cl[i] = p->X[i] - cl[i] / c2;   /* :326-327 */
    double lnl = orc_quadform(p->invcov, cl, p->nused) / 2.0;
    free(cl);
    return lnl;
}

void orc_plik_free(orc_plik_t *p)
{
    if (!p) return;
    for (int s = 0; s < 3; s++) free(p->bins[s]);
    free(p->blmin); free(p->blmax); free(p->weights); free(p->X); free(p->invcov);
    free(p);
}

/* ======================= propose.f90 ======================= */

typedef struct { int n, loopix; int *indices; } orc_cycler_t;   /* CyclicIndexRandomizer */

typedef struct {
    int n, loopix, propose_count;          /* RandDirectionProposer */
    double *R;                             /* n x n row-major, R[j*n+i] = R(j+1,i+1) */
    int block_start;                       /* 1-based */
    int *used_param_indices;               /* n */
    int n_changed;
    int *used_params_changed, *params_changed;   /* n_changed, 1-based */
    double *mapping;                       /* n_changed x n row-major */
} orc_block_t;

struct orc_proposer {
    int nblocks, n_all;
    int *indices, *proposer_for_index;     /* n_all, 1-based values */
    orc_cycler_t slow, fast, all;
    orc_block_t *bp;
    int oversample_fast;
    double propose_scale;
    int fast_ix;
    int n_used;
    int *params_used;
    double *propose_matrix;
};

static int cycler_next(orc_cycler_t *c, orc_rng_t *r)
{   /* propose.f90:75-86 */
    c->loopix = c->loopix % c->n + 1;
    if (c->loopix == 1) {
        if (!c->indices) c->indices = (int *)malloc(sizeof(int) * (size_t)c->n);
        orc_rand_indices(r, c->indices, c->n, c->n);
    }
    return c->indices[c->loopix - 1];
}

orc_proposer_t *orc_proposer_create(int nblocks, const int *block_n, const int *block_params,
                                    int slow_block_max, int oversample_fast, double propose_scale,
                                    int n_used, const int *params_used)
{   /* BlockedProposer Init, propose.f90:151-208 */
    orc_proposer_t *p = (orc_proposer_t *)calloc(1, sizeof(orc_proposer_t));
    p->oversample_fast = oversample_fast;
    p->propose_scale = propose_scale;
    int *used_blocks = (int *)malloc(sizeof(int) * (size_t)nblocks);
    int *block_off = (int *)malloc(sizeof(int) * (size_t)nblocks);
    int n = 0, off = 0;
    for (int i = 0; i < nblocks; i++) {
        block_off[i] = off;
        off += block_n[i];
        if (block_n[i] > 0) {
            p->all.n += block_n[i];
            if (i + 1 <= slow_block_max) p->slow.n += block_n[i];
            used_blocks[n++] = i;
        }
    }
    p->fast.n = p->all.n - p->slow.n;
    p->nblocks = n;
    p->n_all = p->all.n;
    p->bp = (orc_block_t *)calloc((size_t)n, sizeof(orc_block_t));
    p->indices = (int *)calloc((size_t)p->n_all, sizeof(int));
    p->proposer_for_index = (int *)calloc((size_t)p->n_all, sizeof(int));
    int ix = 1;
    for (int i = 0; i < n; i++) {
        orc_block_t *b = &p->bp[i];
        int ub = used_blocks[i];
        b->block_start = ix;
        b->n = block_n[ub];
        b->used_param_indices = (int *)malloc(sizeof(int) * (size_t)b->n);
        for (int k = 0; k < b->n; k++) {
            b->used_param_indices[k] = block_params[block_off[ub] + k];
            p->indices[ix - 1 + k] = b->used_param_indices[k];
            p->proposer_for_index[ix - 1 + k] = i + 1;
        }
        ix += b->n;
    }
    for (int i = 0; i < n; i++) {
        orc_block_t *b = &p->bp[i];
        b->n_changed = p->n_all - b->block_start + 1;
        b->used_params_changed = (int *)malloc(sizeof(int) * (size_t)b->n_changed);
        b->params_changed = (int *)malloc(sizeof(int) * (size_t)b->n_changed);
        for (int k = 0; k < b->n_changed; k++) {
            b->used_params_changed[k] = p->indices[b->block_start - 1 + k];
            b->params_changed[k] = params_used[b->used_params_changed[k] - 1];
        }
        b->R = (double *)calloc((size_t)b->n * b->n, sizeof(double));
        b->mapping = (double *)calloc((size_t)b->n_changed * b->n, sizeof(double));
    }
    p->n_used = n_used;
    p->params_used = (int *)malloc(sizeof(int) * (size_t)n_used);
    memcpy(p->params_used, params_used, sizeof(int) * (size_t)n_used);
    p->propose_matrix = (double *)calloc((size_t)n_used * n_used, sizeof(double));
    free(used_blocks);
    free(block_off);
    return p;
}

void orc_proposer_set_covariance(orc_proposer_t *p, const double *cov)
{   /* BlockedProposer_SetCovariance, propose.f90:210-244 */
    int n = p->n_used;
    memcpy(p->propose_matrix, cov, sizeof(double) * (size_t)n * n);
    double *sig = (double *)malloc(sizeof(double) * (size_t)n);
    double *corr = (double *)malloc(sizeof(double) * (size_t)n * n);
    for (int i = 0; i < n; i++) {
        sig[i] = sqrt(cov[i * n + i]);
        for (int j = 0; j < n; j++) corr[i * n + j] = cov[i * n + j] / sig[i];
    }
    for (int i = 0; i < n; i++)
        for (int k = 0; k < n; k++) corr[k * n + i] = corr[k * n + i] / sig[i];
    int na = p->n_all;
    double *L = (double *)malloc(sizeof(double) * (size_t)na * na);
    for (int i = 0; i < na; i++)
        for (int j = 0; j < na; j++)
            L[i * na + j] = corr[(p->indices[i] - 1) * n + (p->indices[j] - 1)];
    orc_cholesky_lower(L, na);   /* zeroed=.true. */
    for (int i = 0; i < p->nblocks; i++) {
        orc_block_t *b = &p->bp[i];
        for (int j = 0; j < b->n_changed; j++)
            for (int k = 0; k < b->n; k++)
                b->mapping[j * b->n + k] = sig[b->used_params_changed[j] - 1] *
                    L[(b->block_start - 1 + j) * na + (b->block_start - 1 + k)];
    }
    free(sig); free(corr); free(L);
}

static void rot_matrix(orc_rng_t *r, double *M, int n)
{   /* propose.f90:88-102 (propose_rand_directions = .true.) */
    if (n > 1) {
        orc_rand_rotation(r, M, n);
    } else {
        for (int i = 0; i < n * n; i++) M[i] = 0.0;
        for (int i = 0; i < n; i++) M[i * n + i] = (orc_ranmar(r) - 0.5) >= 0.0 ? 1.0 : -1.0;
    }
}

static double propose_r(orc_block_t *b, orc_rng_t *r)
{   /* propose.f90:122-139 */
    if (orc_ranmar(r) < 0.33) return (double)orc_randexp1(r);
    int n = b->n < 2 ? b->n : 2;
    double rf = 0.0;
    for (int i = 0; i < n; i++) {
        double g = orc_gaussian1(r);
        rf += g * g;
    }
    return sqrt(rf / n);
}

static void get_block_proposal(orc_proposer_t *p, orc_rng_t *r, double *P, int i)
{   /* GetBlockProposal :247-254 -> ProposeVec :105-120 -> UpdateParams :142-149 */
    orc_block_t *b = &p->bp[i - 1];
    if (b->loopix % b->n == 0) {
        rot_matrix(r, b->R, b->n);
        b->loopix = 0;
    }
    b->loopix++;
    b->propose_count++;
    double scale = propose_r(b, r) * p->propose_scale;
    double vec[64];
    for (int k = 0; k < b->n; k++) vec[k] = b->R[k * b->n + (b->loopix - 1)] * scale;
    for (int j = 0; j < b->n_changed; j++) {
        double s = 0.0;
        for (int k = 0; k < b->n; k++) s += b->mapping[j * b->n + k] * vec[k];
        P[b->params_changed[j] - 1] += s;
    }
}

void orc_proposer_get_proposal_slow(orc_proposer_t *p, orc_rng_t *r, double *P)
{   /* :275-281 */
    get_block_proposal(p, r, P, p->proposer_for_index[cycler_next(&p->slow, r) - 1]);
}

void orc_proposer_get_proposal_fast(orc_proposer_t *p, orc_rng_t *r, double *P)
{   /* :283-289 */
    get_block_proposal(p, r, P, p->proposer_for_index[p->slow.n + cycler_next(&p->fast, r) - 1]);
}

void orc_proposer_get_proposal(orc_proposer_t *p, orc_rng_t *r, double *P)
{   /* :257-273 */
    if (p->fast_ix != 0) {
        orc_proposer_get_proposal_fast(p, r, P);
        p->fast_ix--;
    } else if (cycler_next(&p->all, r) > p->slow.n) {
        orc_proposer_get_proposal_fast(p, r, P);
        p->fast_ix = p->oversample_fast - 1;
    } else {
        orc_proposer_get_proposal_slow(p, r, P);
    }
}

void orc_proposer_get_proposal_fast_delta(orc_proposer_t *p, orc_rng_t *r, double *P, int num_params)
{   /* :291-298 */
    for (int i = 0; i < num_params; i++) P[i] = 0.0;
    orc_proposer_get_proposal_fast(p, r, P);
}

int orc_proposer_slow_n(const orc_proposer_t *p) { return p->slow.n; }
int orc_proposer_fast_n(const orc_proposer_t *p) { return p->fast.n; }

void orc_proposer_free(orc_proposer_t *p)
{
    if (!p) return;
    for (int i = 0; i < p->nblocks; i++) {
        orc_block_t *b = &p->bp[i];
        free(b->R); free(b->used_param_indices); free(b->used_params_changed);
        free(b->params_changed); free(b->mapping);
    }
    free(p->bp); free(p->indices); free(p->proposer_for_index);
    free(p->slow.indices); free(p->fast.indices); free(p->all.indices);
    free(p->params_used); free(p->propose_matrix);
    free(p);
}

/* ======================= calclike.f90 / MCMC.f90 ======================= */

static void add_like_temp(double *cur, double add, double T)
{   /* calclike.f90:82-94 */
    if (*cur != ORC_LOGZERO) {
        if (add == ORC_LOGZERO) *cur = ORC_LOGZERO;
        else *cur = *cur + add / T;
    }
}

double orc_target_loglike(const orc_target_t *t, const double *P)
{   /* TLikeCalculator GetLogLike, calclike.f90:136-151 */
    double like = 0.0;
    for (int i = 0; i < t->num_params; i++)            /* GetLogLikeBounds :97-109 */
        if (P[i] > t->pmax[i] || P[i] < t->pmin[i]) return ORC_LOGZERO;
    double main = 0.0;
    if (t->test_like) {                                /* TestLikelihoodFunction :180-199 */
        int n = t->n_used;
        double X[64], y[64];
        for (int i = 0; i < n; i++) X[i] = P[t->params_used[i] - 1] - t->center[t->params_used[i] - 1];
        for (int i = 0; i < n; i++) {
            double s = 0.0;
            for (int j = 0; j < n; j++) s += t->test_covinv[i * n + j] * X[j];
            y[i] = s;
        }
        double d = 0.0;
        for (int i = 0; i < n; i++) d += X[i] * y[i];
        main = d / 2.0;
    }
    if (t->plik && t->plik_scale_index > 0) {
        const long n = 3 * t->plik_ld_field;
        double *dl = (double *)malloc((size_t)n * sizeof(double));
        const double a = P[t->plik_scale_index - 1];
        for (long i = 0; i < n; i++) dl[i] = a * t->plik_dl[i];
        main += orc_plik_loglike(t->plik, dl, t->plik_ld_field, P[t->plik_nuis_index - 1]);
        free(dl);
    } else if (t->plik) {
        main += orc_plik_loglike(t->plik, t->plik_dl, t->plik_ld_field, P[t->plik_nuis_index - 1]);
    }
    if (t->extra_like) {                               /* :380-387, the next likelihood of the list */
        const double e = t->extra_like(t->extra_user, P);
        if (e == ORC_LOGZERO) return ORC_LOGZERO;      /* :382 */
        main += e;
    }
    add_like_temp(&like, main, t->temperature);
    if (like == ORC_LOGZERO) return like;
    double pri = 0.0;                                  /* GetLogPriors :111-134 */
    if (t->prior_std)
        for (int i = 0; i < t->num_params; i++)
            if ((!t->varying || t->varying[i] || t->include_fixed_parameter_priors) && t->prior_std[i] != 0.0) {
                double z = (P[i] - t->prior_mean[i]) / t->prior_std[i];
                pri += z * z;
            }
    for (int k = 0; k < t->n_lincomb; k++)             /* :125-131 */
        if (t->lincomb_std[k] != 0.0) {
            const double *w = t->lincomb_weights + (size_t)k * t->num_params;
            double d = 0.0;
            for (int i = 0; i < t->num_params; i++) d += w[i] * P[i];
            double z = (d - t->lincomb_mean[k]) / t->lincomb_std[k];
            pri += z * z;
        }
    pri = pri / 2.0;
    add_like_temp(&like, pri, t->temperature);
    return like;
}

int orc_metropolis_accept(orc_rng_t *r, double like, double cur_like)
{   /* TChainSampler_MetropolisAccept, MCMC.f90:119-131 */
    if (like == ORC_LOGZERO) return 0;
    if (cur_like > like) return 1;
    return (double)orc_randexp1(r) > like - cur_like;
}

int orc_mh_step(orc_proposer_t *prop, orc_rng_t *r, const orc_target_t *t,
                double *P, double *cur_like, int fast_only, double *trial_like_out)
{   /* MCMC.f90:269-307 / 309-335 */
    double trial[256];
    int np = t->num_params;
    memcpy(trial, P, sizeof(double) * (size_t)np);
    if (fast_only) orc_proposer_get_proposal_fast(prop, r, trial);
    else orc_proposer_get_proposal(prop, r, trial);
    double like = orc_target_loglike(t, trial);
    if (trial_like_out) *trial_like_out = like;
    int acc = 0;
    if (like != ORC_LOGZERO) acc = orc_metropolis_accept(r, like, *cur_like);
    if (acc) {
        memcpy(P, trial, sizeof(double) * (size_t)np);
        *cur_like = like;
    }
    return acc;
}

int orc_drag_step(orc_proposer_t *prop, orc_rng_t *r, const orc_target_t *t, orc_drag_state_t *st,
                  double *P, double *cur_like)
{   /* TFastDraggingSampler_GetNewSample, MCMC.f90:338-452 */
    const int np = t->num_params;
    double tend[256], tstart[256], cend[256], cstart[256], delta[256];
    if (*cur_like == ORC_LOGZERO || orc_proposer_fast_n(prop) == 0 || orc_proposer_slow_n(prop) == 0) {
        double tl;                                            /* :351-354 */
        int acc = orc_mh_step(prop, r, t, P, cur_like, 0, &tl);
        st->mult = acc ? 1.0 : st->mult + 1.0;
        return acc;
    }
    st->num_drag++;
    if (st->num_drag % st->oversample_fast != 0) {            /* :357-361 FastParameterSample */
        double tl;
        int acc = orc_mh_step(prop, r, t, P, cur_like, 1, &tl);
        st->mult = acc ? 1.0 : st->mult + 1.0;
        return acc;
    }
    memcpy(tend, P, sizeof(double) * (size_t)np);
    orc_proposer_get_proposal_slow(prop, r, tend);            /* :367-368 */
    double cend_like = orc_target_loglike(t, tend);
    if (cend_like == ORC_LOGZERO) {                           /* :370-374 */
        st->mult += 1.0;
        return 0;
    }
    double cstart_like = *cur_like;
    double sum_e = cend_like, sum_s = cstart_like;
    memcpy(cstart, P, sizeof(double) * (size_t)np);
    memcpy(cend, tend, sizeof(double) * (size_t)np);
    const int nfast = orc_proposer_fast_n(prop);
    int interp = (int)lround(st->dragging_steps * nfast) + 1;   /* :386, nint */
    if (interp < 2) interp = 2;
    for (int is = 1; is <= interp - 1; is++) {
        orc_proposer_get_proposal_fast_delta(prop, r, delta, np);
        for (int i = 0; i < np; i++) tend[i] = cend[i] + delta[i];
        double elike = orc_target_loglike(t, tend), slike = 0.0;
        int acc = elike != ORC_LOGZERO;
        if (acc) {
            for (int i = 0; i < np; i++) tstart[i] = cstart[i] + delta[i];
            slike = orc_target_loglike(t, tstart);
            acc = slike != ORC_LOGZERO;
            if (acc) {
                const double frac = (double)is / interp;
                const double cint = cstart_like * (1 - frac) + frac * cend_like;
                const double ilike = slike * (1 - frac) + frac * elike;
                acc = orc_metropolis_accept(r, ilike, cint);
            }
        }
        if (acc) {
            memcpy(cend, tend, sizeof(double) * (size_t)np);
            memcpy(cstart, tstart, sizeof(double) * (size_t)np);
            cend_like = elike;
            cstart_like = slike;
        }
        sum_s = sum_s + cstart_like;
        sum_e = sum_e + cend_like;
    }
    const double cur_drag = sum_s / interp, drag = sum_e / interp;
    int acc = orc_metropolis_accept(r, drag, cur_drag);       /* :436 */
    if (acc) {
        memcpy(P, cend, sizeof(double) * (size_t)np);
        *cur_like = cend_like;
        st->mult = 1.0;
    } else {
        st->mult += 1.0;
    }
    return acc;
}

/* ======================= samples.f90 ======================= */

static void jacobi_eigenvalues(double *A, int n, double *ev)
{   /* symmetric eigenvalues (stands in for DSYEV's values; order-independent use) */
    for (int sweep = 0; sweep < 100; sweep++) {
        double off = 0.0;
        for (int i = 0; i < n; i++)
            for (int j = i + 1; j < n; j++) off += A[i * n + j] * A[i * n + j];
        if (off < 1e-30) break;
        for (int p = 0; p < n; p++)
            for (int q = p + 1; q < n; q++) {
                double apq = A[p * n + q];
                if (fabs(apq) < 1e-300) continue;
                double theta = (A[q * n + q] - A[p * n + p]) / (2.0 * apq);
                double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < n; k++) {
                    double akp = A[k * n + p], akq = A[k * n + q];
                    A[k * n + p] = c * akp - s * akq;
                    A[k * n + q] = s * akp + c * akq;
                }
                for (int k = 0; k < n; k++) {
                    double apk = A[p * n + k], aqk = A[q * n + k];
                    A[p * n + k] = c * apk - s * aqk;
                    A[q * n + k] = s * apk + c * aqk;
                }
            }
    }
    for (int i = 0; i < n; i++) ev[i] = A[i * n + i];
}

double orc_gelman_rubin(const double *cov, const double *meanscov, int n)
{   /* GelmanRubinEvalues, samples.f90:41-67; returns maxval(evals) */
    double *rot = (double *)malloc(sizeof(double) * (size_t)n * n);
    double *rm = (double *)malloc(sizeof(double) * (size_t)n * n);
    double *T = (double *)malloc(sizeof(double) * (size_t)n * n);
    double *ev = (double *)malloc(sizeof(double) * (size_t)n);
    memcpy(rot, cov, sizeof(double) * (size_t)n * n);
    memcpy(rm, meanscov, sizeof(double) * (size_t)n * n);
    for (int jj = 0; jj < n; jj++) {
        double sc = sqrt(cov[jj * n + jj]);
        for (int k = 0; k < n; k++) { rot[jj * n + k] /= sc; rm[jj * n + k] /= sc; }
        for (int k = 0; k < n; k++) { rot[k * n + jj] /= sc; rm[k * n + jj] /= sc; }
    }
    double R = 1e6;
    if (orc_cholesky_lower(rot, n) == 0) {           /* Matrix_CholeskyRootInverse */
        lower_inverse(rot, n);
        for (int i = 0; i < n; i++)                   /* rot * rm */
            for (int j = 0; j < n; j++) {
                double s = 0.0;
                for (int k = 0; k < n; k++) s += rot[i * n + k] * rm[k * n + j];
                T[i * n + j] = s;
            }
        for (int i = 0; i < n; i++)                   /* (rot*rm) * rot^T */
            for (int j = 0; j < n; j++) {
                double s = 0.0;
                for (int k = 0; k < n; k++) s += T[i * n + k] * rot[j * n + k];
                rm[i * n + j] = s;
            }
        jacobi_eigenvalues(rm, n, ev);
        R = ev[0];
        for (int i = 1; i < n; i++) if (ev[i] > R) R = ev[i];
    }
    free(rot); free(rm); free(T); free(ev);
    return R;
}
