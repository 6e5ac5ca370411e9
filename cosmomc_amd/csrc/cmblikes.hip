// CMBlikes bandpower likelihoods (reference TCMBLikes, source/CMBlikes.f90)
// and the BICEP/Keck/Planck foreground model (TBK_planck,
// source/CMB_BK_Planck.f90), batched over W walkers on MI355X.
//
// Per walker (CMBLikes_LogLike, CMBlikes.f90:1165-1227):
//   map spectra  MapCl_ij(l) = Theory_{f_i f_j}(l) [+ aberration] [+ foregrounds] [/ cal^2]
//                                             (GetTheoryMapCls / AdaptTheoryForMaps :1022-1126)
//   binning      Cls(out, b) = sum_win dot(W(:,win,b), MapCl_in(win))  [+ linear correction]
//                                             (TBinWindows_bin :1230-1256, GetBinnedMapCls :981-995)
//   per bin      C = Cls (+ noise);  HL:  X_b = Transform(C, Chat_b, Cfid_b^1/2)   (:861-914)
//                                    gaussian: X_b = C - Chat_b
//   -lnL         = (bigX^T C^-1 bigX + (ln cal / sigma)^2) / 2         (:1220-1225)
//
// Kernels:
//   cmbl_bk_prologue        BK foreground SEDs and l profiles per walker
//   cmbl_window_direct /    every window column as a dot product with one map
//   cmbl_window_kernel /    spectrum: a skinny f64 MFMA GEMM over l chunks
//   cmbl_window_group       (grouped map pairs for the BK foregrounds)
//   cmbl_gauss_small_kernel gaussian datasets with <= 64 bandpowers: chi^2 in one kernel
//   cmbl_reduce_kernel      binned C matrices / bigX rows
//   cmbl_hl_rows_kernel<M>  the HL transform per (walker, bin): two symmetric
//                           eigendecompositions by one-sided (Hestenes) cyclic Jacobi
//   cmbl_exact_kernel       like_approx = exact (unbinned): ExactChiSq per (walker, l)
//   quadform_ksplit         bigX^T C^-1 bigX / 2 on the f64 MFMA (quadform.hip).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <set>
#include <sstream>

#include "divrn.h"
#include "quadform.h"
#include "smallgauss.h"

namespace cmamd {

static constexpr int CL_MAXMAPS = 16;          // HL matrices up to 16 x 16 in one wave
static constexpr int CL_MAXREQ = 32;            // required maps
static constexpr int BK_NPARAM = 16;            // BKPlanck.paramnames
static constexpr int WK_COLS = 32;              // window columns per work item (two 16-row MFMA blocks)
static constexpr int WK_CHUNK = 64;             // l per chunk
#ifndef CMAMD_WK_NCH
#define CMAMD_WK_NCH 4
#endif
static constexpr int WK_NCH = CMAMD_WK_NCH;     // chunks per work item
static constexpr int WK_TS = WK_CHUNK + 2;      // LDS row stride of the spectrum tile (doubles)

typedef double f64x4 __attribute__((ext_vector_type(4)));

struct CLPair {      // one required map pair (i >= j)
    int field;       // theory field index 0..9 (TT TE EE BT BE BB PT PE PB PP)
    int cmb;         // both theory indices <= B: aberration and calibration apply
    int fg;          // foregrounds: 0 none, 1 BK EE, 2 BK BB, 3 SMICA TT
    int mi, mj;      // required-map indices (0-based)
};

struct WItem {       // one (map pair, <= WK_NCH l chunks, <= WK_COLS window columns) contraction
    int pair;
    int l0, l1;      // l range (inclusive), l0 even when possible
    int ncol;
    int part;        // partial rows part .. part+ncol-1
    int nch;         // chunks of WK_CHUNK l
    long long woff;  // dense weights [nch][WK_CHUNK][WK_COLS] (zero padded)
    long long woff2; // direct-kernel weights [nch][ncol blocks][16 columns][WK_CHUNK] (zero padded)
};

struct BKMap {       // per required map: bandpass samples and constants (Read_Bandpass :72-105)
    int off, n;      // samples in bp_nu / bp_R / bp_dnu
    int bc;          // band-centre error slot: 0 none, 1 '95', 2 '150', 3 '220'
    int pad;
    double th_dust, th_sync, nu_bar;
};

struct CLDev {
    int lmin, lmax;                 // pcl_lmin, pcl_lmax
    int nitem;
    const WItem *items;
    const double *wdense;
    const double *wdirect;
    const CLPair *pairs;
    double aberration;
    int cal_index;                  // 0-based in DataParams, -1 none
    double log_cal_prior;           // > 0: add (ln cal / prior)^2 to chi^2
    // reduction to binned spectra, per element e = bin * ncl + cl
    int nE, ncl_used, nX, Np, approx, has_corr;
    const int *e_main_off, *e_main_rows, *e_corr_off, *e_corr_rows;   // partial rows per element
    const double *e_main_const, *e_corr_const;   // fixed-spectrum (fix_cl) window dots per element
    const double *fidcorr;          // [nE]
    const double *noise;            // [nE] (HL)
    const double *chat;             // [nE] (gaussian)
    const int *e_to_x;              // [nE] gaussian: index into bigX or -1
    // BK foregrounds
    int bk, nreq;
    int LP;                         // profile row length: prof[w][3][LP], indexed by l (zero outside lmin..lmax)
                                    // (SMICA: prof[w][0] = A1 exp(..), prof[w][1] = A2 (l/pivot)^n2)
    double smica_pivot;             // TSmica_planck%pivot (CMBlikes.f90:1270)
    const BKMap *bkmaps;
    const double *bp_nu, *bp_R, *bp_dnu;
    const double *bp_lnu;           // log(nu) of every bandpass sample
    int nsamp;                      // bandpass samples, all maps
    double *td_den;                 // [nsamp] exp(G nu / Td0) - 1 for the launch's first walker's Td0 (cmbl_bk_tdtab);
    double *td0;                    // [1] that Td0.  Both live in the call's workspace, so launches on other
                                    // streams with their own workspaces never share the table
    const double *log_l80;          // log(l / 80), l = 0 .. LP-1
    double fpivot_dust, fpivot_sync, decorr_dust[2], decorr_sync[2];
    int lform_dust, lform_sync;     // 0 flat, 1 lin, 2 quad
    // sparse evaluation (the sampler's per-likelihood change mask): walkers
    // [0, *wcount) of the launch are live, the rest exit; null = all W
    const int *wcount;
};

// live walkers of a launch over W (wcount: device count, or null)
__device__ __forceinline__ int live_walkers(const int *wcount, int W) { return wcount ? min(W, *wcount) : W; }

static constexpr double BK_TCMB = 2.72548;
static constexpr double BK_H = 6.62606957e-34;
static constexpr double BK_KB = 1.3806488e-23;
__host__ __device__ inline double ghz_kelvin() { return BK_H / BK_KB * 1e9; }

__device__ inline double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// Decorrelation (CMB_BK_Planck.f90:187-227)
__device__ inline double bk_decorr(double Delta, double nu0, double nu1, const double *piv, int l, int lform) {
    const double lpivot = 80.0;
    const double a = log(nu0 / nu1), b = log(piv[0] / piv[1]);
    const double scl_nu = (a * a) / (b * b);
    double scl_ell = 1.0;
    if (lform == 1) scl_ell = l / lpivot;
    else if (lform == 2) {
        const double t = l / lpivot;
        scl_ell = t * t;
    }
    if (Delta > 1.0) return 2.0 - exp(log(2.0 - Delta) * scl_nu * scl_ell);
    return exp(log(Delta) * scl_nu * scl_ell);
}

// The dust greybody's denominators exp(G nu / T_dust) - 1 of every bandpass
// sample at the first walker's T_dust (a fixed parameter in the BK15 runs, so
// every walker's): cmbl_bk_prologue takes them from here when its walker's
// T_dust is the same value -- the same operations, so the same bits -- and
// forms them itself otherwise.  One of its three exponentials per sample.
__global__ __launch_bounds__(256) void cmbl_bk_tdtab(CLDev c, const double *__restrict__ nuis)
{
    const double Tdust = nuis[4];   // DataParams(5) of walker 0 (row 0 exists whenever a prologue runs)
    const double G = ghz_kelvin();
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k < c.nsamp) c.td_den[k] = exp(G * c.bp_nu[k] / Tdust) - 1;
    if (k == 0) c.td0[0] = Tdust;
}

// BK per-walker foreground set-up (TBK_planck_AddForegrounds :250-285): the
// SED factors of every map (one wave per map, bandpass integrals as wave
// reductions) and the dust / sync / dust-sync l profiles.
//   coef[w][3][nreq] = fdust, fsync, band-centre error;  prof[w][3][L]
#ifndef CMAMD_BKP_THREADS
#define CMAMD_BKP_THREADS 256
#endif
static constexpr int BKP_THREADS = CMAMD_BKP_THREADS;   // a wave per map at a time
__global__ __launch_bounds__(BKP_THREADS) void cmbl_bk_prologue(CLDev c, const double *__restrict__ nuis, long long ld_nuis,
                                                       double *__restrict__ coef, double *__restrict__ prof, int W)
{
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int w = blockIdx.x;
    if (w >= live_walkers(c.wcount, W)) return;
    const double *P = nuis + (long long)w * ld_nuis;
    const double Adust = P[0], Async = P[1], alphadust = P[2], betadust = P[3], Tdust = P[4];
    const double alphasync = P[5], betasync = P[6], dustsync_corr = P[7];
    const double G = ghz_kelvin();
    double *cw = coef + (long long)w * 3 * c.nreq;
    // pivot-frequency SEDs: the same for every map of this walker, so computed once
    const double nu0d = c.fpivot_dust, nu0s = c.fpivot_sync;
    const double gb0 = pow(nu0d, 3 + betadust) / (exp(G * nu0d / Tdust) - 1);
    const double pl0 = pow(nu0s, 2 + betasync);
    const bool tab = Tdust == c.td0[0];              // cmbl_bk_tdtab's denominators apply
    for (int i = wave; i < c.nreq; i += BKP_THREADS / 64) {
        const BKMap m = c.bkmaps[i];
        double gb = 0.0, pl = 0.0;
        for (int k = lane; k < m.n; k += 64) {
            const double nu = c.bp_nu[m.off + k], R = c.bp_R[m.off + k], dn = c.bp_dnu[m.off + k];
            const double lnu = c.bp_lnu[m.off + k];          // nu^e as exp(e log nu): one exp instead of a pow
            const double den = tab ? c.td_den[m.off + k] : exp(G * nu / Tdust) - 1;
            gb += dn * R * exp((3 + betadust) * lnu) / den;
            pl += dn * R * exp((2 + betasync) * lnu);
        }
        gb = wave_sum(gb);
        pl = wave_sum(pl);
        if (lane == 0) {
            double bc = 1.0;
            if (m.bc == 1) bc = P[12] + P[13] + 1.;
            else if (m.bc == 2) bc = P[12] + P[14] + 1.;
            else if (m.bc == 3) bc = P[12] + P[15] + 1.;
            double th_err = 1.0, gb_err = 1.0, pl_err = 1.0;
            if (bc != 1.) {                                   // DustScaling :130-141, SyncScaling :169-178
                const double e1 = exp(G * m.nu_bar / BK_TCMB) - 1, e2 = exp(G * m.nu_bar * bc / BK_TCMB) - 1;
                th_err = (bc * bc * bc * bc) * exp(G * m.nu_bar * (bc - 1) / BK_TCMB) * (e1 * e1) / (e2 * e2);
                gb_err = pow(bc, 3 + betadust) * (exp(G * m.nu_bar / Tdust) - 1) / (exp(G * m.nu_bar * bc / Tdust) - 1);
                pl_err = pow(bc, 2 + betasync);
            }
            cw[i] = (gb / gb0) / m.th_dust * (gb_err / th_err);
            cw[c.nreq + i] = (pl / pl0) / m.th_sync * (pl_err / th_err);
            cw[2 * c.nreq + i] = bc;
        }
    }
    const int LP = c.LP;
    double *pw = prof + (long long)w * 3 * LP;
    for (int l = tid; l < LP; l += blockDim.x) {
        if (l < c.lmin || l > c.lmax) {
            pw[l] = pw[LP + l] = pw[2 * LP + l] = 0.0;
            continue;
        }
        const double ll = c.log_l80[l];                     // (l/80)^a as exp(a log(l/80))
        pw[l] = Adust * exp(alphadust * ll);
        pw[LP + l] = Async * exp(alphasync * ll);
        pw[2 * LP + l] = dustsync_corr * sqrt(Adust * Async) * exp(((alphadust + alphasync) / 2) * ll);
    }
}

// SMICA's TT foreground (TSmica_planck_AddForegrounds, CMBlikes.f90:1295-1322)
// per walker and l as two profile rows, added to every TT map pair in window
// staging in the reference's order: (D_l + A1 exp(n1 lnr + n1run/2 lnr^2)) +
// A2 (l/pivot)^n2, lnr = ln(l/pivot).  prof[w][3][LP]; row 2 unused.
__global__ __launch_bounds__(256) void cmbl_smica_prologue(CLDev c, const double *__restrict__ nuis, long long ld_nuis,
                                                          double *__restrict__ prof, int W)
{
    const int w = blockIdx.y;
    if (w >= live_walkers(c.wcount, W)) return;
    const int l = blockIdx.x * 256 + threadIdx.x;
    const int LP = c.LP;
    if (l >= LP) return;
    const double *P = nuis + (long long)w * ld_nuis;
    double *pw = prof + (long long)w * 3 * LP;
    if (l < c.lmin || l > c.lmax) {
        pw[l] = pw[LP + l] = 0.0;
        return;
    }
    const double A1 = P[0], n1 = P[1], n1run = P[2], A2 = P[3], n2 = P[4];
    const double x = (double)l / c.smica_pivot;
    const double lnrat = log(x);
    pw[l] = A1 * exp(n1 * lnrat + n1run / 2 * (lnrat * lnrat));
    pw[LP + l] = A2 * pow(x, n2);
}

// TSmica_planck_derivedParameters (CMBlikes.f90:1324-1337): derived(1) =
// Cls(1,1)%CL(2000) of map cross-spectra initialised to zero plus the
// foregrounds, i.e. the TT foreground at l = 2000 when the first required map
// pair is TT (0 otherwise); any further derived columns 0 (the base
// TDataLikelihood_derivedParameters, GeneralTypes.f90:504-512).  NaN when
// l = 2000 is outside pcl_lmin..pcl_lmax (the reference reads out of bounds).
__global__ __launch_bounds__(64) void cmbl_smica_derived(CLDev c, int tt11, const double *__restrict__ nuis,
                                                        long long ld_nuis, double *__restrict__ out, long long ld_out,
                                                        int nd, int W)
{
    const int w = blockIdx.x * 64 + threadIdx.x;
    if (w >= W) return;
    const double *P = nuis + (long long)w * ld_nuis;
    double *o = out + (long long)w * ld_out;
    const int l = 2000;
    double v = 0.0;
    if (l < c.lmin || l > c.lmax) v = __builtin_nan("");
    else if (tt11) {
        const double A1 = P[0], n1 = P[1], n1run = P[2], A2 = P[3], n2 = P[4];
        const double x = (double)l / c.smica_pivot;
        const double lnrat = log(x);
        v = (v + A1 * exp(n1 * lnrat + n1run / 2 * (lnrat * lnrat))) + A2 * pow(x, n2);
    }
    o[0] = v;
    for (int k = 1; k < nd; k++) o[k] = 0.0;
}

// Window contractions on the f64 MFMA.  One workgroup = 64 walkers x one work
// item (map pair, up to WK_NCH chunks of WK_CHUNK l, <= WK_COLS window columns):
//   partial[col][w] = sum_l Wt[l][col] MapCl_w(l)
// The walkers' map spectra MapCl_w(l) (GetTheoryMapCls + AdaptTheoryForMaps,
// CMBlikes.f90:1022-1126: aberration, foregrounds, calibration) are formed
// while staging each theory chunk into LDS from coalesced 16-byte row loads;
// the next chunk's loads are in flight during the current chunk's MFMAs.
// Each wave owns 16 walkers: v_mfma_f64_16x16x4f64 over (column block, 4 l).
// ABER / FG (the dataset's aberration / foreground switches) are template
// parameters so the lensing variant carries no foreground code.
template <bool ABER, bool FG>
__global__ __launch_bounds__(256) void cmbl_window_kernel(CLDev c, const double *__restrict__ dl, long long ld_field,
                                                         long long ld_walker, const double *__restrict__ nuis,
                                                         long long ld_nuis, const double *__restrict__ coef,
                                                         const double *__restrict__ prof, double *__restrict__ partial,
                                                         int W, int vec_ok)
{
    __shared__ __attribute__((aligned(16))) double wsh[WK_CHUNK * WK_COLS];   // weights [l][col]
    __shared__ __attribute__((aligned(16))) double tsh[64 * WK_TS];           // spectra [walker][l]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int w0 = blockIdx.x * 64;
    const int Wc = live_walkers(c.wcount, W);
    if (w0 >= Wc) return;
    const WItem it = c.items[blockIdx.y];
    const CLPair pr = c.pairs[it.pair];
    const bool aber = ABER && c.aberration != 0.0 && pr.cmb;
    const bool fg = FG && pr.fg;
    // staging map: thread -> l pair q = tid % 32 of rows r_u = tid / 32 + 8 u (u < 8)
    constexpr int PER = 64 * (WK_CHUNK / 2) / 256;
    const int q = tid % (WK_CHUNK / 2), rbase = tid / (WK_CHUNK / 2);
    // per-walker constants of the thread's rows
    double calsq[PER];
    double dust[FG ? PER : 1], sync[FG ? PER : 1], dsync[FG ? PER : 1], ddf[FG ? PER : 1], dsf[FG ? PER : 1],
        nui[FG ? PER : 1], nuj[FG ? PER : 1], Ddust[FG ? PER : 1], Dsync[FG ? PER : 1];
    bool dd_l = false, ds_l = false;     // l-dependent decorrelation (lform lin / quad) in use
#pragma unroll
    for (int u = 0; u < PER; u++) {
        const int w = min(w0 + rbase + 8 * u, Wc - 1);
        const double *P = nuis + (long long)w * ld_nuis;
        const double cl = c.cal_index >= 0 ? P[c.cal_index] : 1.0;
        calsq[u] = cl * cl;
        if constexpr (FG) {
            dust[u] = sync[u] = dsync[u] = nui[u] = nuj[u] = 0.0;
            ddf[u] = dsf[u] = Ddust[u] = Dsync[u] = 1.0;
            if (fg && pr.fg != 3) {                           // :296-328
                const double *cw = coef + (long long)w * 3 * c.nreq;
                const int a = pr.mi, b = pr.mj;
                double d = cw[a] * cw[b], sy = cw[c.nreq + a] * cw[c.nreq + b];
                double ds = cw[a] * cw[c.nreq + b] + cw[c.nreq + a] * cw[b];
                if (pr.fg == 1) {
                    const double EEd = P[8], EEs = P[9];
                    d = d * EEd;
                    sy = sy * EEs;
                    ds = ds * sqrt(EEd * EEs);
                }
                dust[u] = d;
                sync[u] = sy;
                dsync[u] = ds;
                const double Delta_dust = P[10], Delta_sync = P[11];
                Ddust[u] = Delta_dust;
                Dsync[u] = Delta_sync;
                nui[u] = c.bkmaps[a].nu_bar * cw[2 * c.nreq + a];
                nuj[u] = c.bkmaps[b].nu_bar * cw[2 * c.nreq + b];
                // need_dust_decorr .and. i /= j (:288-289, :312); flat l-scaling is one factor per pair
                if (fabs(Delta_dust - 1) > 1e-5 && a != b) {
                    if (c.lform_dust == 0) ddf[u] = bk_decorr(Delta_dust, nui[u], nuj[u], c.decorr_dust, 0, 0);
                    else dd_l = true;
                } else {
                    Ddust[u] = 1.0;   // marks "no decorrelation" for this walker
                }
                if (fabs(Delta_sync - 1) > 1e-5 && a != b) {
                    if (c.lform_sync == 0) dsf[u] = bk_decorr(Delta_sync, nui[u], nuj[u], c.decorr_sync, 0, 0);
                    else ds_l = true;
                } else {
                    Dsync[u] = 1.0;
                }
            }
        }
    }
    double2 raw[PER];
    auto load_chunk = [&](int ch) {
        const int lq = it.l0 + ch * WK_CHUNK + 2 * q;
#pragma unroll
        for (int u = 0; u < PER; u++) {
            const int w = w0 + rbase + 8 * u;
            raw[u] = make_double2(0.0, 0.0);
            if (w < Wc && lq <= it.l1) {
                const double *Df = dl + (long long)w * ld_walker + (long long)pr.field * ld_field;
                if (vec_ok) {
                    raw[u] = *reinterpret_cast<const double2 *>(Df + lq);
                } else {
                    raw[u].x = Df[lq];
                    if (lq + 1 <= it.l1) raw[u].y = Df[lq + 1];
                }
            }
        }
    };
    f64x4 acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
    const int li = lane & 15, lk = lane >> 4;
    const double *trow = tsh + (16 * wave + li) * WK_TS;
    load_chunk(0);
    for (int ch = 0; ch < it.nch; ch++) {
        {   // weights of this chunk (zero-padded to WK_COLS columns and WK_CHUNK l by the host)
            const double2 *src = reinterpret_cast<const double2 *>(c.wdense + it.woff) + ch * (WK_CHUNK * WK_COLS / 2);
            for (int i = tid; i < WK_CHUNK * WK_COLS / 2; i += 256) reinterpret_cast<double2 *>(wsh)[i] = src[i];
        }
        const int lq = it.l0 + ch * WK_CHUNK + 2 * q;
#pragma unroll
        for (int u = 0; u < PER; u++) {
            const int r = rbase + 8 * u, w = w0 + r;
            double v2[2] = {raw[u].x, raw[u].y};
            if (w < Wc && lq <= it.l1) {
                const double *Df = dl + (long long)w * ld_walker + (long long)pr.field * ld_field;
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const int l = lq + h;
                    if (l > it.l1) break;
                    double v = v2[h];
                    if (aber) {                               // AddAberration :1062-1101
                        int la = l - 1, lb = l + 1;
                        if (l == c.lmin) { la = l; lb = l + 2; }
                        else if (l == c.lmax) { la = l - 2; lb = l; }
                        const double ea = la, eb = lb, el = l;
                        const double ca = Df[la] / (ea * (ea + 1)), cb = Df[lb] / (eb * (eb + 1));
                        const double deriv = 0.5 * (cb - ca);
                        v = v + c.aberration * (el * el * (el + 1) * deriv);
                    }
                    if constexpr (FG) {
                        if (fg && pr.fg == 3) {               // SMICA TT (CMBlikes.f90:1314-1317)
                            const double *pw = prof + (long long)w * 3 * c.LP + l;
                            v = v + pw[0];
                            v = v + pw[c.LP];
                        } else if (fg) {                      // :329-334
                            const double *pw = prof + (long long)w * 3 * c.LP + l;
                            const double Dd = (dd_l && Ddust[u] != 1.0)
                                                  ? bk_decorr(Ddust[u], nui[u], nuj[u], c.decorr_dust, l, c.lform_dust)
                                                  : ddf[u];
                            const double Ds = (ds_l && Dsync[u] != 1.0)
                                                  ? bk_decorr(Dsync[u], nui[u], nuj[u], c.decorr_sync, l, c.lform_sync)
                                                  : dsf[u];
                            v = v + dust[u] * pw[0] * Dd + sync[u] * pw[c.LP] * Ds + dsync[u] * pw[2 * c.LP];
                        }
                    }
                    if (c.cal_index >= 0 && pr.cmb) v = v / calsq[u];   // AdaptTheoryForMaps :1113-1124
                    v2[h] = v;
                }
            }
            tsh[r * WK_TS + 2 * q] = v2[0];
            tsh[r * WK_TS + 2 * q + 1] = v2[1];
        }
        if (ch + 1 < it.nch) load_chunk(ch + 1);          // in flight during this chunk's MFMAs
        __syncthreads();
        // A = Wt[col][k] (lane: col = lane&15, k = lane>>4); B = MapCl[k][walker] (walker = lane&15)
        const int clen = min(WK_CHUNK, it.l1 - (it.l0 + ch * WK_CHUNK) + 1);
        const int nk = (clen + 3) / 4;
        if (it.ncol > 16) {
            for (int s = 0; s < nk; s++) {
                const int k = 4 * s + lk;
                const double b = trow[k];
                const double a0 = wsh[k * WK_COLS + li];
                const double a1 = wsh[k * WK_COLS + 16 + li];
                acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b, acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b, acc1, 0, 0, 0);
            }
        } else {                                            // one 16-column block suffices
            for (int s = 0; s < nk; s++) {
                const int k = 4 * s + lk;
                acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(wsh[k * WK_COLS + li], trow[k], acc0, 0, 0, 0);
            }
        }
        __syncthreads();
    }
    // D: walker = lane&15, col = (lane>>4) + 4 r
    const int w = w0 + 16 * wave + li;
    if (w < Wc) {
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int c0 = lk + 4 * r, c1 = 16 + lk + 4 * r;
            if (c0 < it.ncol) partial[(long long)(it.part + c0) * W + w] = acc0[r];
            if (c1 < it.ncol) partial[(long long)(it.part + c1) * W + w] = acc1[r];
        }
    }
}

// Window contraction without aberration or foregrounds (TBinWindows_bin
// :1230-1256 on GetTheoryMapCls :1022-1052).  The spectrum operand comes
// straight from global memory: lane (walker li, quarter kq) of a wave holds the
// 8 l {l0 + 32 st + 8 j + 2 kq + h : j < 4, h < 2} of its walker's spectrum in
// slot 2 j + h, and MFMA step s = 2 j + h contracts the four l {8 j + 2 kq + h};
// every load is a 16-byte vector, and the four kq lanes of a walker read 64
// contiguous bytes per load instruction (one half line, not four scattered
// quarters), and the next step's spectra are in flight during this step's MFMAs.  The weights
// (8 KB per 64 l) are shared by the block's four waves through a
// double-buffered LDS tile: read per wave from L2 they cost 24.2 vs 17.7 us per
// launch (lensing, W = 1024, MI355X).  The calibration (AdaptTheoryForMaps
// :1113-1124, D_l / cal^2 for T/E/B pairs) is linear and is applied to the
// sums.  Blocks are dealt to the 8 XCDs round-robin; the remap puts all walker
// tiles of an item on one XCD so its weights are fetched into one L2 (17.9 vs
// 18.7 us with the linear order; 17.5 vs 17.7 us against an XCD-balanced split).
__global__ __launch_bounds__(256) void cmbl_window_direct(CLDev c, const double *__restrict__ dl, long long ld_field,
                                                         long long ld_walker, const double *__restrict__ nuis,
                                                         long long ld_nuis, double *__restrict__ partial, int W,
                                                         int tiles, int vec_ok)
{
    constexpr int LPL = 8, STEP = 4 * LPL, NSUB = WK_CHUNK / STEP, WROW = STEP + 2;
    __shared__ __attribute__((aligned(16))) double wsh[2 * 2 * 16 * WROW];   // [buf][col block][col][l]
    // blocks are dealt to the XCDs round-robin: all walker tiles of an item on one XCD
    // (its weights in one L2); measured faster than an XCD-balanced split of the units
    const int b = blockIdx.x, xcd = b & 7, j = b >> 3;
    const int item = xcd + 8 * (j / tiles), tile = j % tiles;
    if (item >= c.nitem) return;
    const int Wc = live_walkers(c.wcount, W);
    if (tile * 64 >= Wc) return;
    const WItem it = c.items[item];
    const CLPair pr = c.pairs[it.pair];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int li = lane & 15, kq = lane >> 4;
    const int w = tile * 64 + wave * 16 + li;
    const int wl = min(w, Wc - 1);
    const double *Df = dl + (long long)wl * ld_walker + (long long)pr.field * ld_field;
    const int ncb = (it.ncol + 15) >> 4;
    const int nstep = it.nch * NSUB;
    double t[LPL], tn[LPL], tnn[LPL], a[LPL], a2[LPL];
    static_assert(LPL == 8, "slot 2 j + h holds l = 8 j + 2 kq + h");
    auto load_t = [&](int st, double *dst) {
        const int lb = it.l0 + st * STEP + 2 * kq;
        if (vec_ok && it.l0 + st * STEP + STEP - 1 <= it.l1) {
#pragma unroll
            for (int j = 0; j < LPL / 2; j++) {
                const double2 v = *reinterpret_cast<const double2 *>(Df + lb + 8 * j);
                dst[2 * j] = v.x;
                dst[2 * j + 1] = v.y;
            }
        } else {
#pragma unroll
            for (int j = 0; j < LPL / 2; j++)
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const int l = lb + 8 * j + h;
                    dst[2 * j + h] = (l <= it.l1) ? Df[l] : 0.0;
                }
        }
    };
    // weights [nch][ncb][16][WK_CHUNK]; thread tid moves column tid/16, l 2 (tid%16) .. +1
    auto wsrc = [&](int st, int cb) {
        const int ch = st / NSUB, sub = st % NSUB;
        return c.wdirect + it.woff2 + ((long long)ch * ncb + cb) * 16 * WK_CHUNK + sub * STEP;
    };
    const int wc = tid >> 4, wp = 2 * (tid & 15);
    double2 wr0, wr1;
    auto fetch_w = [&](int st) {
        wr0 = *reinterpret_cast<const double2 *>(wsrc(st, 0) + wc * WK_CHUNK + wp);
        if (ncb > 1) wr1 = *reinterpret_cast<const double2 *>(wsrc(st, 1) + wc * WK_CHUNK + wp);
    };
    auto store_w = [&](int buf) {
        *reinterpret_cast<double2 *>(wsh + ((buf * 2 + 0) * 16 + wc) * WROW + wp) = wr0;
        if (ncb > 1) *reinterpret_cast<double2 *>(wsh + ((buf * 2 + 1) * 16 + wc) * WROW + wp) = wr1;
    };
    auto read_w = [&](int buf, int cb, double *dst) {   // A operand: column li at the lane's LPL l
        const double *src = wsh + ((buf * 2 + cb) * 16 + li) * WROW + 2 * kq;
#pragma unroll
        for (int j = 0; j < LPL / 2; j++) {
            const double2 v = *reinterpret_cast<const double2 *>(src + 8 * j);
            dst[2 * j] = v.x;
            dst[2 * j + 1] = v.y;
        }
    };
    f64x4 acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
    // the spectra run two steps ahead (measured neutral: the read pattern itself
    // gives 4.2-4.5 TB/s here with the MFMAs removed, tools/membench2.hip 6.2)
    load_t(0, t);
    fetch_w(0);
    if (nstep > 1) load_t(1, tn);
    store_w(0);
    __syncthreads();
    for (int st = 0; st < nstep; st++) {
        const bool more = st + 1 < nstep;
        const int cur = st & 1;
        if (more) fetch_w(st + 1);                     // in flight across this step's MFMAs
        if (st + 2 < nstep) load_t(st + 2, tnn);
        read_w(cur, 0, a);
        if (ncb > 1) read_w(cur, 1, a2);
#pragma unroll
        for (int s = 0; s < LPL; s++) acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], t[s], acc0, 0, 0, 0);
        if (ncb > 1) {
#pragma unroll
            for (int s = 0; s < LPL; s++) acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a2[s], t[s], acc1, 0, 0, 0);
        }
        if (more) {
            store_w(cur ^ 1);      // buffer cur ^ 1 was last read before the previous barrier
            __syncthreads();
#pragma unroll
            for (int s = 0; s < LPL; s++) {
                t[s] = tn[s];
                tn[s] = tnn[s];
            }
        }
    }
    if (w < Wc) {
        double inv = 1.0;
        if (c.cal_index >= 0 && pr.cmb) {
            const double cl = nuis[(long long)w * ld_nuis + c.cal_index];
            inv = cl * cl;
        }
        // D: walker = lane&15, column = (lane>>4) + 4 r
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int c0 = kq + 4 * r, c1 = 16 + kq + 4 * r;
            if (c0 < it.ncol) partial[(long long)(it.part + c0) * W + w] = acc0[r] / inv;
            if (c1 < it.ncol) partial[(long long)(it.part + c1) * W + w] = acc1[r] / inv;
        }
    }
}

// BK foreground datasets (TBK_planck, CMB_BK_Planck.f90:229-340): every map pair
// p of a theory field reads the same four per-walker rows -- the theory D_l and
// the dust / sync / dust-sync l profiles of cmbl_bk_prologue -- and differs only
// in per-(pair, walker) SED coefficients:
//   MapCl_p(l) = D_l + (dust_p Pd(l) Dd_p(l) + sync_p Ps(l) Ds_p(l) + dsync_p Px(l))
// (the expression of cmbl_window_kernel's staging, :329-334 of the reference).
// A work item is (up to GP pairs of one field, <= GSEG l); the workgroup
// (64 walkers, 16 per wave) loads each lane's 4 consecutive l of the four rows
// once per 16-l step and forms every pair's MapCl in registers for
// v_mfma_f64_16x16x4f64 against that pair's <= 16 window columns, so a row
// element is read once per item instead of once per pair (78 B x B pairs for
// BK15).  l-dependent decorrelation (lform lin / quad with Delta /= 1) is
// evaluated per value, as in the staged kernel.
#ifndef CMAMD_GP
#define CMAMD_GP 8
#endif
#ifndef CMAMD_GSEG
#define CMAMD_GSEG 224
#endif
// l per grouped item: 224 (BK15's l range in three items a pair group),
// cmbl_window_group 85.8 -> 78.1 us and configs[4] 396.4-397.8 -> 388.2-390.3
// us/step, against 160 / 192 / 256 / 320 / 608 (406 / 417-418 / 397 / 412-414 /
// 441 us/step; tools/gpu_r6m.sh); 6 pairs per item 400-401
static constexpr int GP = CMAMD_GP;       // pairs per grouped item
static constexpr int GSEG = CMAMD_GSEG;   // l per grouped item (a multiple of 32)
static_assert(GSEG % 32 == 0, "grouped items are whole 32-l steps");
static_assert((GP * 16 * 16 / 2) % 256 == 0, "the weight staging moves GP * 16 rows of 16 l in whole passes");

struct GItem {
    int field, npair, l0, nstep;
    int pair[GP];       // CLPair index
    int ncol[GP];       // columns of each pair (<= 16)
    int part[GP];       // first partial row of each pair
    long long woff;     // weights [GP][16][nstep * 32] (zero padded)
};

// LDEC: l-dependent decorrelation possible (lform_dust or lform_sync lin / quad);
// without it no pair's flags can be set, and the inner loop carries no
// decorrelation code (same arithmetic on the flags = 0 path)
template <bool LDEC>
__global__ __launch_bounds__(256, 2) void cmbl_window_group(CLDev c, const GItem *__restrict__ gitems, int ngitem,
                                                        const double *__restrict__ wts, const double *__restrict__ dl,
                                                        long long ld_field, long long ld_walker,
                                                        const double *__restrict__ nuis, long long ld_nuis,
                                                        const double *__restrict__ coef, const double *__restrict__ prof,
                                                        int LP, double *__restrict__ partial, int W, int tiles,
                                                        int vec_ok, int tile_xcd)
{
    constexpr int LPL = 4, STEP = 4 * LPL;
    // per-(pair, walker) SED coefficients: [GP][8][64] = dust, sync, dsync, ddf, dsf, nui, nuj, flags
    __shared__ double cf[GP][8][64];
    // the item's window weights of one step, double-buffered: [GP * 16 columns][STEP (+2 pad)]
    constexpr int WR = STEP + 2;
    __shared__ __attribute__((aligned(16))) double wsh[2][GP * 16 * WR];
    // blocks are dealt to the XCDs round-robin.  tile_xcd (tiles % 8 == 0): each XCD
    // owns tiles / 8 walker tiles and runs every item for them, so a walker's four
    // rows are fetched into one L2 (the items of one l segment re-read them once per
    // pair group); else all walker tiles of an item on one XCD (its weights in one L2)
    const int b = blockIdx.x, xcd = b & 7, j = b >> 3;
    int item, tile;
    if (tile_xcd) {
        const int tpx = tiles >> 3;
        tile = xcd + 8 * (j % tpx);
        item = j / tpx;
    } else {
        item = xcd + 8 * (j / tiles);
        tile = j % tiles;
    }
    if (item >= ngitem) return;
    const int Wc = live_walkers(c.wcount, W);
    if (tile * 64 >= Wc) return;
    const GItem &it = gitems[item];
    const int np = it.npair;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    {   // staged kernel :226-258, one (walker, pair) per thread and pass
        const int ws = min(tile * 64 + lane, Wc - 1);
        const double *P = nuis + (long long)ws * ld_nuis;
        const double *cw = coef + (long long)ws * 3 * c.nreq;
        const double Delta_dust = P[10], Delta_sync = P[11];
        for (int g = wave; g < np; g += 4) {
            const CLPair pr = c.pairs[it.pair[g]];
            double d = 0.0, sy = 0.0, ds = 0.0, ddf = 1.0, dsf = 1.0, nui = 0.0, nuj = 0.0;
            int flags = 0;
            if (pr.fg) {
                const int a = pr.mi, bb = pr.mj;
                d = cw[a] * cw[bb];
                sy = cw[c.nreq + a] * cw[c.nreq + bb];
                ds = cw[a] * cw[c.nreq + bb] + cw[c.nreq + a] * cw[bb];
                if (pr.fg == 1) {
                    const double EEd = P[8], EEs = P[9];
                    d = d * EEd;
                    sy = sy * EEs;
                    ds = ds * sqrt(EEd * EEs);
                }
                nui = c.bkmaps[a].nu_bar * cw[2 * c.nreq + a];
                nuj = c.bkmaps[bb].nu_bar * cw[2 * c.nreq + bb];
                if (fabs(Delta_dust - 1) > 1e-5 && a != bb) {
                    if (c.lform_dust == 0) ddf = bk_decorr(Delta_dust, nui, nuj, c.decorr_dust, 0, 0);
                    else flags |= 1;
                }
                if (fabs(Delta_sync - 1) > 1e-5 && a != bb) {
                    if (c.lform_sync == 0) dsf = bk_decorr(Delta_sync, nui, nuj, c.decorr_sync, 0, 0);
                    else flags |= 2;
                }
            }
            cf[g][0][lane] = d;
            cf[g][1][lane] = sy;
            cf[g][2][lane] = ds;
            cf[g][3][lane] = ddf;
            cf[g][4][lane] = dsf;
            cf[g][5][lane] = nui;
            cf[g][6][lane] = nuj;
            cf[g][7][lane] = (double)flags;
        }
    }
    const int li = lane & 15, kq = lane >> 4;
    const int wr_ = wave * 16 + li;                // walker within the tile
    const int w = tile * 64 + wr_;
    const int wl = min(w, Wc - 1);
    const double *P = nuis + (long long)wl * ld_nuis;
    const double Delta_dust = P[10], Delta_sync = P[11];
    const double *Df = dl + (long long)wl * ld_walker + (long long)it.field * ld_field;
    const double *pw = prof + (long long)wl * 3 * LP;
    double t[4][LPL], tn[4][LPL];
    auto load = [&](int st, double (*dst)[LPL]) {
        const int lb = it.l0 + st * STEP + LPL * kq;
        if (vec_ok && lb + LPL - 1 <= c.lmax) {
#pragma unroll
            for (int s = 0; s < LPL / 2; s++) {
                const double2 v0 = reinterpret_cast<const double2 *>(Df + lb)[s];
                const double2 v1 = reinterpret_cast<const double2 *>(pw + lb)[s];
                const double2 v2 = reinterpret_cast<const double2 *>(pw + LP + lb)[s];
                const double2 v3 = reinterpret_cast<const double2 *>(pw + 2 * LP + lb)[s];
                dst[0][2 * s] = v0.x; dst[0][2 * s + 1] = v0.y;
                dst[1][2 * s] = v1.x; dst[1][2 * s + 1] = v1.y;
                dst[2][2 * s] = v2.x; dst[2][2 * s + 1] = v2.y;
                dst[3][2 * s] = v3.x; dst[3][2 * s + 1] = v3.y;
            }
        } else {
#pragma unroll
            for (int s = 0; s < LPL; s++) {
                const int l = lb + s;
                const bool ok = l <= c.lmax;
                dst[0][s] = ok ? Df[l] : 0.0;
                dst[1][s] = ok ? pw[l] : 0.0;
                dst[2][s] = ok ? pw[LP + l] : 0.0;
                dst[3][s] = ok ? pw[2 * LP + l] : 0.0;
            }
        }
    };
    f64x4 acc[GP];
#pragma unroll
    for (int g = 0; g < GP; g++) acc[g] = f64x4{0.0, 0.0, 0.0, 0.0};
    const int Lp = it.nstep * 32;
    const int nst = it.nstep * (32 / STEP);
    // weights of step st: GP*16 rows of STEP doubles; thread q moves rows q / (STEP/2) ...
    constexpr int NW2 = GP * 16 * STEP / 2, PERT = NW2 / 256;
    double2 wr[PERT];
    auto fetch_w = [&](int st) {
#pragma unroll
        for (int u = 0; u < PERT; u++) {
            const int q = tid + 256 * u, row = q / (STEP / 2), c2 = q % (STEP / 2);
            wr[u] = row < np * 16 ? reinterpret_cast<const double2 *>(wts + it.woff + (long long)row * Lp + st * STEP)[c2]
                                  : make_double2(0.0, 0.0);
        }
    };
    auto store_w = [&](int buf) {
#pragma unroll
        for (int u = 0; u < PERT; u++) {
            const int q = tid + 256 * u, row = q / (STEP / 2), c2 = q % (STEP / 2);
            *reinterpret_cast<double2 *>(&wsh[buf][row * WR + 2 * c2]) = wr[u];
        }
    };
    load(0, t);
    fetch_w(0);
    store_w(0);
    __syncthreads();
    for (int st = 0; st < nst; st++) {
        const bool more = st + 1 < nst;
        const int cur = st & 1;
        if (more) {                                    // in flight across this step's MFMAs
            load(st + 1, tn);
            fetch_w(st + 1);
        }
        const int lr = st * STEP + LPL * kq;
#pragma unroll
        for (int g = 0; g < GP; g++) {
            if (g >= np) break;
            const double *src = &wsh[cur][(g * 16 + li) * WR + LPL * kq];
            const double2 q0 = reinterpret_cast<const double2 *>(src)[0], q1 = reinterpret_cast<const double2 *>(src)[1];
            const double a[LPL] = {q0.x, q0.y, q1.x, q1.y};
            const double dg = cf[g][0][wr_], sg = cf[g][1][wr_], xg = cf[g][2][wr_];
            const int flags = (int)cf[g][7][wr_];
#pragma unroll
            for (int s = 0; s < LPL; s++) {
                double Dd = cf[g][3][wr_], Ds = cf[g][4][wr_];
                if (LDEC && flags) {
                    const int l = it.l0 + lr + s;
                    if (flags & 1) Dd = bk_decorr(Delta_dust, cf[g][5][wr_], cf[g][6][wr_], c.decorr_dust, l, c.lform_dust);
                    if (flags & 2) Ds = bk_decorr(Delta_sync, cf[g][5][wr_], cf[g][6][wr_], c.decorr_sync, l, c.lform_sync);
                }
                const double v = t[0][s] + (dg * t[1][s] * Dd + sg * t[2][s] * Ds + xg * t[3][s]);
                acc[g] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], v, acc[g], 0, 0, 0);
            }
        }
        if (more) {
            store_w(cur ^ 1);          // buffer cur ^ 1 was last read before the previous barrier
            __syncthreads();
#pragma unroll
            for (int q = 0; q < 4; q++)
#pragma unroll
                for (int s = 0; s < LPL; s++) t[q][s] = tn[q][s];
        }
    }
    if (w < Wc) {
#pragma unroll
        for (int g = 0; g < GP; g++) {
            if (g >= np) break;
            double inv = 1.0;
            if (c.cal_index >= 0 && c.pairs[it.pair[g]].cmb) {
                const double cl = P[c.cal_index];
                inv = cl * cl;
            }
            // D: walker = lane & 15, column = (lane >> 4) + 4 r
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int col = kq + 4 * r;
                if (col < it.ncol[g]) partial[(long long)(it.part[g] + col) * W + w] = acc[g][r] / inv;
            }
        }
    }
}

// Binned spectra per (walker, element e = bin * ncl + cl): window columns in
// window order (TBinWindows_bin :1230-1256), each column the l-chunk partials
// in order, plus the linear correction (GetBinnedMapCls :981-995).  Gaussian:
// writes bigX = C - Chat for the used spectra; HL: writes C (+ noise) for the
// transform.  Block (0, 0) zeroes the quadratic-form tickets; element 0 also
// pads the bigX row and writes the calibration-prior addend.
__global__ __launch_bounds__(256) void cmbl_reduce_kernel(CLDev c, const double *__restrict__ partial,
                                                         const double *__restrict__ nuis, long long ld_nuis,
                                                         double *__restrict__ xrows, double *__restrict__ cmat,
                                                         double *__restrict__ addend, unsigned int *__restrict__ counters,
                                                         int n_counters, int W)
{
    // a workgroup is 64 walkers x four elements, one per wave (BK15's 702 elements
    // have 3 partial rows each: 702 x 16 four-wave workgroups, three waves of each
    // mostly idle, took 11.8 us)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int e = blockIdx.y * 4 + wave;
    const int w = blockIdx.x * 64 + lane;
    if (blockIdx.x == 0 && blockIdx.y == 0)
        for (int i = threadIdx.x; i < n_counters; i += 256) counters[i] = 0u;
    const int Wc = live_walkers(c.wcount, W);
    if (blockIdx.x * 64 >= Wc || e >= c.nE) return;
    // window columns in window order, each the l-chunk partials in order (flattened on
    // the host); four interleaved sums k over rows k, k+4, ... eight loads at a time,
    // combined in fixed order: deterministic (and the order the earlier four-wave
    // form had, wave k taking sum k)
    auto rows_sum = [&](const int *off, const int *rows) {
        double v[4] = {0.0, 0.0, 0.0, 0.0};
        if (w < Wc) {
            const int q0 = off[e], q1 = off[e + 1];
#pragma unroll
            for (int k = 0; k < 4; k++)
                for (int q = q0 + k; q < q1; q += 32) {
                    double t[8];
#pragma unroll
                    for (int u = 0; u < 8; u++)
                        t[u] = (q + 4 * u < q1) ? partial[(long long)rows[q + 4 * u] * W + w] : 0.0;
#pragma unroll
                    for (int u = 0; u < 8; u++) v[k] += t[u];
                }
        }
        return ((v[0] + v[1]) + v[2]) + v[3];
    };
    const double main = rows_sum(c.e_main_off, c.e_main_rows);
    const double corr = c.has_corr ? rows_sum(c.e_corr_off, c.e_corr_rows) : 0.0;
    if (w >= Wc) return;
    double s = c.e_main_const[e] + main;
    if (c.has_corr) {
        const double cs = c.e_corr_const[e] + corr;
        s = s + (cs - c.fidcorr[e]);
    }
    double *x = xrows + (long long)w * c.Np;
    if (c.approx == 2) {
        const int ix = c.e_to_x[e];
        if (ix >= 0) x[ix] = s - c.chat[e];
    } else {
        cmat[(long long)w * c.nE + e] = s + c.noise[e];
    }
    if (e == 0) {
        for (int k = c.nX; k < c.Np; k++) x[k] = 0.0;
        if (addend) {
            double a = 0.0;
            if (c.log_cal_prior > 0 && c.cal_index >= 0) {
                const double t = log(nuis[(long long)w * ld_nuis + c.cal_index]) / c.log_cal_prior;
                a = t * t / 2;
            }
            addend[w] = a;
        }
    }
}

// Small gaussian likelihoods (nX <= 64, e.g. lensing 9, SPT-SZ 47): the
// whole chi^2 in one kernel (smallgauss.h).  The host cuts the partial rows of
// every element into tasks of <= 8 rows.
struct SmallTask { int first, count; };      // rows e_*_rows[first .. first+count) (host side)
struct SmallDev {
    int ntask;
    const int *trow;                         // [ntask][8]: each task's partial rows, -1 padded
    const int *e_main_t, *e_corr_t;          // [nE+1] task ranges per element
};

template <int WT>
__global__ __launch_bounds__(256) void cmbl_gauss_small_kernel(SmallGaussLaunch a, int ng)
{
    __shared__ double lds[small_gauss_lds_doubles<WT>()];
    const int q = small_gauss_group(blockIdx.x, ng);
    if (q < ng) small_gauss_body<WT>(a, lds, q);
}

// ---------------------------------------------------------------- HL
struct HLDev {
    int n, m, nb, ncl, ncl_used, nX, Np;
    const double *chat;     // [nb][n][n]
    const double *cfhalf;   // [nb][n][n]
    const double *u0;       // [nb][n][n] eigenvectors (columns) of C_fid: the first eigensolve's starting basis
    const double *v0;       // [nb][n][n] eigenvectors of C_fid^-1/2 Chat C_fid^-1/2: the second's
    const int *cl_use;
    int *status;            // sticky CMBL_STATUS_* bits (cmbl_status)
    const int *wcount;      // live walkers (CLDev::wcount)
};

// ------------------------------------------- HL, register-resident (M lanes / matrix)
// The two symmetric eigensolves and HL transform of CMBLikes_Transform
// (:861-914) by one-sided cyclic Jacobi (hl_ojacobi), with the matrices in
// registers: lane r of an M-lane group owns column r of the working matrix
// and of the eigenvector matrix, and a 64-lane block packs 64/M (walker, bin)
// problems.  The matrix products go through per-group LDS row buffers.
#ifdef CMAMD_STAMPS
__device__ unsigned int g_hl_sweeps[2][64];      // waves per sweep count, first / second eigensolve (tools/hl_stamps.py)
// s_memtime ticks per Jacobi round phase, summed over the rounds of lane 0 of
// every wave: [0] column write + barrier, [1] partner read, dot product and
// angle, [2] rotation + barrier, [3] rounds
__device__ unsigned long long g_hl_phase[4];
// s_memtime ticks per kernel phase, summed over lane 0 of every wave (tools/hl_stamps.py)
__device__ unsigned long long g_hl_tp[12];
#define HL_STAMP(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#else
#define HL_STAMP(v) ((void)0)
#endif

// one problem's buffers; per-problem strides of 2 mod 32 LDS dwords put the
// groups' broadcast reads of one element on distinct bank pairs (at 16 mod 32,
// BK15's M = 12, groups 0, 2 and 4 shared a pair: 3-way conflicts)
template <int M>
struct HLGrpLds {
    static constexpr int SZ = 2 * M * (M + 1) + 2 * M;          // doubles before the pad
    double rows[2][M][M + 1];       // two row buffers (odd stride: fewer bank conflicts within a problem);
                                    // in the Jacobi, buffer 1 holds each row as of the round start
    double dg[M];                   // a diagonal / g(x) broadcast
    double isd[M];                  // 1 / sqrt of the first eigensolve's eigenvalues
    double pad[((1 - SZ) % 16 + 16) % 16 + 1];
};

template <int M>
struct HLRowsLds {
    static constexpr int G = 64 / M;   // problems per wave: M lanes each, packed (5 for M = 12)
    HLGrpLds<M> g[G];
};

template <int M>
__device__ inline int hl_partner(int rr, int r) {   // round-robin pairing of round rr (circle method)
    if (r == M - 1) return rr;
    if (r == rr) return M - 1;
    return ((2 * rr - r) % (M - 1) + (M - 1)) % (M - 1);
}

static constexpr int HL_MAX_SWEEPS = 40;
// a sweep in which no pair of a problem was further from orthogonal than
// cos = 1e-6 is that problem's last (its own rotations leave every pair near
// cos 1e-12: -lnL within 2.4e-14 relative of the reference's DSYEV on the BK
// goldens, tools/hl_margin.py).  With the stop per problem a looser one buys
// little, since a wave runs until its slowest problem stops: BK15 at W = 1024
// HL 173.7 / 170.9 / 167.5 us at cos 1e-6 / 1e-5 / 1e-4, golden margins
// 2.4e-14 / 2.3e-12 / 2.1e-10, and cos 1e-4 fails the 9-map width test's
// rtol 1e-9 (round 5, profiles/r05_hl_stop.txt)
#ifndef CMAMD_HL_SWEEP_COS2
#define CMAMD_HL_SWEEP_COS2 1e-12
#endif
static constexpr double HL_SWEEP_COS2 = CMAMD_HL_SWEEP_COS2;
#ifndef CMAMD_HL_VFREE
#define CMAMD_HL_VFREE 1
#endif
static constexpr bool HL_VFREE = CMAMD_HL_VFREE;   // as DSYEV's own iteration limit, a cap that fails loudly

// One-sided (Hestenes) cyclic Jacobi of the group's symmetric M x M matrix C:
// lane r owns column r of G (initially C's column r, i.e. its row r) and
// column r of V (initially e_r).  A round pairs lanes (lo, hi) by the
// round-robin circle schedule; both lanes of a pair read the other's columns
// from LDS, form a_ll = g_l.g_l, a_hh = g_h.g_h, a_lh = g_l.g_h (the same sums
// in the same order, so both derive the same rotation) and rotate their own
// columns: g_l' = c g_l - s g_h, g_h' = s g_l + c g_h, with tan of the angle
// the smaller root of t^2 + 2 zeta t - 1 = 0, zeta = (a_hh - a_ll) / (2 a_lh).
// At convergence G = C V and V holds orthonormal eigenvectors in its columns;
// lam = v_r . g_r = v_r^T C v_r is eigenvalue r, signed.  One column exchange
// per round (two barriers) replaces the two-sided form's row exchange plus
// broadcast of every column's rotation (three barriers, about twice the LDS
// traffic); the column norms are carried across rounds, so a round forms one
// dot product, and the arithmetic is fused multiply-adds (the eigensolver is
// not the reference's DSYEV, so no operation order is there to follow).  Pairs
// with |a_lh| > 1e-15 sqrt(a_ll a_hh) are rotated; a sweep in which no pair of
// a problem had |a_lh| > 1e-6 sqrt(a_ll a_hh) (HL_SWEEP_COS2 = 1e-12 on the
// squares) ends that problem's solve (its own rotations, by the quadratic
// convergence of cyclic Jacobi, leave every pair near 1e-12: no separate check
// sweep).  The stop is per problem: a problem whose sweep met it rotates no
// more while the other problems of its wave go on, so its result depends on
// its own matrix only, not on which walkers share its wave.
// Returns true on lanes whose pair still needed rotating in sweep
// HL_MAX_SWEEPS (the caller fails that problem: NaN and a status bit).
// VF (V-free): the matrices here are symmetric positive definite (C, and
// C^-1/2 Chat C^-1/2), so G = C V = U Sigma with U = V: eigenvalue r is the
// norm of column r and eigenvector r that column normalised, and V need not
// be carried -- each round exchanges and rotates one column instead of two
// (the exchange is the round's cost: lane permutes through the LDS crossbar).
template <int M, bool VF = false>
__device__ bool hl_ojacobi(double (&G)[M], double (&V)[M], HLRowsLds<M> &S, int grp, int r, int lane, int which,
                           double &lam)
{
    (void)which;
    (void)lane;
    const bool on = grp < HLRowsLds<M>::G;        // lanes past G*M idle
    if (!VF)
#pragma unroll
        for (int k = 0; k < M; k++) V[k] = (k == r) ? 1.0 : 0.0;
    if (VF) {   // the input matrix (row r = column r), for the eigenvalues' signs after the solve
        if (on)
#pragma unroll
            for (int k = 0; k < M; k++) S.g[grp].rows[0][r][k] = G[k];
        __syncthreads();
    }
    bool failed = false;
    bool done = !on;                              // this lane's problem has met the sweep stop
    const unsigned long long gmask = (M == 64 ? ~0ull : ((1ull << M) - 1)) << ((on ? grp : 0) * M);
#ifdef CMAMD_STAMPS
    unsigned long long ph0 = 0, ph1 = 0, ph2 = 0, nround = 0;
#endif
    for (int sweep = 0;; sweep++) {
        bool big = false;
        // the column's squared norm, recomputed every sweep and updated exactly
        // as Rutishauser's a_ll' = a_ll - t a_lh, a_hh' = a_hh + t a_lh in between
        double nrm = 0.0;
#pragma unroll
        for (int k = 0; k < M; k++) nrm = fma(G[k], G[k], nrm);
#pragma unroll 1
        for (int rr = 0; rr < M - 1; rr++) {
            const int p = on ? hl_partner<M>(rr, r) : r;
            HL_STAMP(t0);
            // the partner's column and norm by lane permutes (ds_bpermute: no LDS
            // banks, no barrier; the same values the row buffers carried)
            const int src = on ? grp * M + p : lane;
            HL_STAMP(t1);
#ifdef CMAMD_STAMPS
            unsigned long long t2 = 0;
#endif
            double Gp[M], Vp[M];
#pragma unroll
            for (int k = 0; k < M; k++) {        // every permute in flight together
                Gp[k] = __shfl(G[k], src);
                if (!VF) Vp[k] = __shfl(V[k], src);
            }
            const double np_ = __shfl(nrm, src);
            if (!done) {
                const bool low = r < p;
                const double all = low ? nrm : np_, ahh = low ? np_ : nrm;
                double alh = 0.0;
#pragma unroll
                for (int k = 0; k < M; k++) alh = fma(low ? G[k] : Gp[k], low ? Gp[k] : G[k], alh);
                if (alh != 0.0 && alh * alh > 1e-30 * (all * ahh)) {
                    // cos^2 > HL_SWEEP_COS2: columns this far from orthogonal need another
                    // sweep; below it this sweep's rotation leaves them near cos^2 squared
                    big = big || alh * alh > HL_SWEEP_COS2 * (all * ahh);
                    const double d = ahh - all, e = 2.0 * alh;
                    // the hardware square root (not correctly rounded): den only sets the
                    // angle, and c, s stay orthonormal to rounding whatever t is
                    const double den = fabs(d) + __builtin_amdgcn_sqrt(d * d + e * e);
                    const double q = __builtin_amdgcn_rcp(den);     // the hardware reciprocal: likewise
                    const double t = ((d >= 0) == (e >= 0) ? fabs(e) : -fabs(e)) * q;
                    const double c = rsqrt(t * t + 1.0), s = t * c;
#ifdef CMAMD_STAMPS
                    t2 = __builtin_amdgcn_s_memtime();
#endif
                    if (low) {
#pragma unroll
                        for (int k = 0; k < M; k++) {
                            G[k] = fma(-s, Gp[k], c * G[k]);
                            if (!VF) V[k] = fma(-s, Vp[k], c * V[k]);
                        }
                        nrm = fma(-t, alh, all);
                    } else {
#pragma unroll
                        for (int k = 0; k < M; k++) {
                            G[k] = fma(s, Gp[k], c * G[k]);
                            if (!VF) V[k] = fma(s, Vp[k], c * V[k]);
                        }
                        nrm = fma(t, alh, ahh);
                    }
                }
            }
#ifdef CMAMD_STAMPS
            {
                const unsigned long long t3 = __builtin_amdgcn_s_memtime();
                const unsigned long long t2w = __shfl(t2, 0) ? __shfl(t2, 0) : t3;
                ph0 += t1 - t0;
                ph1 += t2w - t1;
                ph2 += t3 - t2w;
                nround++;
            }
#endif
        }
#ifdef CMAMD_STAMPS
        if (!__any(big) || sweep == HL_MAX_SWEEPS)
            if (lane == 0) atomicAdd(&g_hl_sweeps[which][sweep < 63 ? sweep : 63], 1u);
#endif
        // per problem: a sweep with no big pair is its last (wave-uniform exit once
        // every problem of the wave is done)
        const unsigned long long bal = __ballot(big);
        if (!(bal & gmask)) done = true;
        if (!bal) break;
        if (sweep == HL_MAX_SWEEPS) {
            failed = big;
            break;
        }
    }
#ifdef CMAMD_STAMPS
    if (lane == 0) {
        atomicAdd(&g_hl_phase[0], ph0);
        atomicAdd(&g_hl_phase[1], ph1);
        atomicAdd(&g_hl_phase[2], ph2);
        atomicAdd(&g_hl_phase[3], nround);
    }
#endif
    if (VF) {
        double n2 = 0.0;
#pragma unroll
        for (int k = 0; k < M; k++) n2 = fma(G[k], G[k], n2);
        const double sg = sqrt(n2), rsg = 1.0 / sg;
#pragma unroll
        for (int k = 0; k < M; k++) V[k] = n2 > 0.0 ? div_rn(G[k], sg, rsg) : (k == r ? 1.0 : 0.0);   // G[k] / sg
        // |g_r| is |lambda_r| and g_r / |g_r| is sign(lambda_r) u_r, so the norm alone
        // loses the sign of an eigenvalue of a matrix that is not positive definite
        // (a trial theory C can be): lambda_r = (A v)_i / v_i at the largest |v_i|,
        // so a negative eigenvalue stays negative and its sqrt / log give NaN, as the
        // reference's DSYEV eigenvalues do (CMBlikes.f90:877-894)
        int im = 0;
        double vm = V[0];
#pragma unroll
        for (int k = 1; k < M; k++)
            if (fabs(V[k]) > fabs(vm)) {
                im = k;
                vm = V[k];
            }
        double d = 0.0;
        if (on)
#pragma unroll
            for (int k = 0; k < M; k++) d = fma(S.g[grp].rows[0][im][k], V[k], d);
        __syncthreads();   // the callers reuse the row buffers
        lam = (d * vm < 0.0) ? -sg : sg;
        return failed;
    }
    double l = 0.0;
#pragma unroll
    for (int k = 0; k < M; k++) l = fma(V[k], G[k], l);
    lam = l;
    return failed;
}

template <int M>
__global__ __launch_bounds__(64, (M <= 12 ? 2 : 1)) void cmbl_hl_rows_kernel(HLDev h, const double *__restrict__ cmat,
                                                         double *__restrict__ xrows, int W)
{
    __shared__ HLRowsLds<M> S;
    constexpr int G = HLRowsLds<M>::G;
    const int lane = threadIdx.x, grp = lane / M, r = lane % M;
    const bool on = grp < G;                      // lanes past G*M idle
    const int prob = blockIdx.x * G + grp;
    const int nprob = live_walkers(h.wcount, W) * h.nb;
    if (blockIdx.x * G >= nprob) return;          // block-uniform: no live problem
    const bool live = on && prob < nprob;
    const int w = live ? prob / h.nb : 0, b = live ? prob % h.nb : 0;
    const int n = h.n;
    const bool row_ok = on && r < n;
    auto U_row = [&](int k, int j) { return S.g[grp].rows[0][k][j]; };
    // C row r from its lower-triangle elements (ElementsToMatrix :950-965), zero padded to M
    HL_STAMP(q0);
    double A[M], V[M];
    const double *cm = cmat + ((long long)w * h.nb + b) * h.ncl;
#pragma unroll
    for (int j = 0; j < M; j++) {
        double v = 0.0;
        if (live && row_ok && j < n) {
            const int a = r > j ? r : j, bb = r > j ? j : r;
            v = cm[a * (a + 1) / 2 + bb];
        }
        A[j] = v;
    }
    // Warm start: the solve runs on B0^T A B0, with B0 the eigenvectors of
    // the fiducial's matrix (host, per bin), which is nearly diagonal for
    // walkers near the fiducial, and maps its eigenvectors back (V <- B0 V).
    // Lane r holds row r of A (= column r); B0 rows go to row buffer 1.
    auto to_basis = [&](const double *B0) {
        if (on)
#pragma unroll
            for (int k = 0; k < M; k++) S.g[grp].rows[1][r][k] = (row_ok && k < n) ? B0[r * n + k] : (k == r ? 1.0 : 0.0);
        __syncthreads();
        double T[M];
#pragma unroll
        for (int j = 0; j < M; j++) {             // T = A B0, row r
            double s = 0.0;
#pragma unroll
            for (int k = 0; k < M; k++) s += A[k] * S.g[grp].rows[1][k][j];
            T[j] = s;
        }
        if (on)
#pragma unroll
            for (int k = 0; k < M; k++) S.g[grp].rows[0][r][k] = T[k];
        __syncthreads();
#pragma unroll
        for (int j = 0; j < M; j++) {             // B0^T T, row r
            double s = 0.0;
#pragma unroll
            for (int k = 0; k < M; k++) s += S.g[grp].rows[1][k][r] * S.g[grp].rows[0][k][j];
            A[j] = s;
        }
        __syncthreads();
    };
    auto from_basis = [&]() {                     // V <- B0 V (column r), B0 still in row buffer 1
        double U[M];
#pragma unroll
        for (int i = 0; i < M; i++) {
            double s = 0.0;
#pragma unroll
            for (int k = 0; k < M; k++) s += S.g[grp].rows[1][i][k] * V[k];
            U[i] = s;
        }
#pragma unroll
        for (int i = 0; i < M; i++) V[i] = U[i];
        __syncthreads();
    };
    // (1) C = U diag U^T (lane r: eigenvector r, i.e. column r of U)
    double dgr;
#ifdef CMAMD_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    HL_STAMP(q1);
    if (h.u0) to_basis(h.u0 + (long long)b * n * n);
    HL_STAMP(q2);
    bool unconverged = hl_ojacobi<M, HL_VFREE>(A, V, S, grp, r, lane, 0, dgr);
    HL_STAMP(q3);
    if (h.u0) from_basis();
    if (on) {
        S.g[grp].dg[r] = dgr;
        S.g[grp].isd[r] = 1.0 / sqrt(dgr);
#pragma unroll
        for (int k = 0; k < M; k++) S.g[grp].rows[0][k][r] = V[k];     // U rows, from its columns
    }
    __syncthreads();
    // (2) T = Chat U ; R = U^T T scaled by 1/sqrt(diag) (:878-889)
    // row r of Chat (and below of Cfhalf) into registers first, every load in
    // flight together (a runtime-n loop waited on each load in turn); the sums
    // keep the k order
    double T[M], hr[M];
    const double *ch = h.chat + (long long)b * n * n;
#pragma unroll
    for (int k = 0; k < M; k++) hr[k] = (row_ok && k < n) ? ch[r * n + k] : 0.0;
#pragma unroll
    for (int j = 0; j < M; j++) {
        double s = 0.0;
        if (row_ok && j < n)
#pragma unroll
            for (int k = 0; k < M; k++)
                if (k < n) s += hr[k] * U_row(k, j);
        T[j] = s;
    }
    if (on)
#pragma unroll
        for (int k = 0; k < M; k++) S.g[grp].rows[1][r][k] = T[k];
    __syncthreads();
    double R[M];
#pragma unroll
    for (int j = 0; j < M; j++) {
        double s = 0.0;
        if (row_ok && j < n) {
#pragma unroll
            for (int k = 0; k < M; k++)
                if (k < n) s += U_row(k, r) * S.g[grp].rows[1][k][j];
            const int lo = r < j ? r : j, hi = r < j ? j : r;
            s = s * S.g[grp].isd[lo] * S.g[grp].isd[hi];   // the reference divides by each root (:886-889)
        }
        R[j] = s;
    }
    __syncthreads();
    HL_STAMP(q4);
    // (3) Rot = U R U^T (:891): T2 = R U^T (rows through LDS), A = U T2
    if (on)
#pragma unroll
        for (int k = 0; k < M; k++) S.g[grp].rows[1][r][k] = R[k];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < M; j++) {        // T2[r][j] = sum_k R[r][k] U[j][k]
        double s = 0.0;
        if (row_ok && j < n)
#pragma unroll
            for (int k = 0; k < M; k++)
                if (k < n) s += R[k] * U_row(j, k);
        T[j] = s;
    }
    __syncthreads();
    if (on)
#pragma unroll
        for (int k = 0; k < M; k++) S.g[grp].rows[1][r][k] = T[k];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < M; j++) {        // A[r][j] = sum_k U[r][k] T2[k][j]
        double s = 0.0;
        if (row_ok && j < n)
#pragma unroll
            for (int k = 0; k < M; k++)
                if (k < n) s += U_row(r, k) * S.g[grp].rows[1][k][j];
        A[j] = s;
    }
    __syncthreads();
    // (4) Rot = V diag V^T; g(x) = sign(x - 1) sqrt(2 max(0, x - ln x - 1))  (:892-894)
    double x;
    HL_STAMP(q5);
    if (h.v0) to_basis(h.v0 + (long long)b * n * n);
    HL_STAMP(q6);
    unconverged = hl_ojacobi<M, HL_VFREE>(A, V, S, grp, r, lane, 1, x) || unconverged;
    HL_STAMP(q7);
    if (h.v0) from_basis();
    __syncthreads();                               // the solve's last reads of the row buffers
    if (on) {
        // a NaN argument (x < 0 or NaN: a C that is not positive definite) stays NaN:
        // fmax(0, NaN) would make it 0 and the point's chi^2 finite
        const double arg = x - log(x) - 1;
        const double g = arg == arg ? sqrt(2 * fmax(0.0, arg)) : arg;
        S.g[grp].dg[r] = (x - 1 >= 0) ? g : -g;
#pragma unroll
        for (int k = 0; k < M; k++) S.g[grp].rows[0][k][r] = V[k];     // V rows, from its columns
    }
    __syncthreads();
    HL_STAMP(q8);
    // (5) U = Cfhalf V ; C = U diag(g) U^T (:907-912)
    const double *cf = h.cfhalf + (long long)b * n * n;
#pragma unroll
    for (int k = 0; k < M; k++) hr[k] = (row_ok && k < n) ? cf[r * n + k] : 0.0;
#pragma unroll
    for (int j = 0; j < M; j++) {
        double s = 0.0;
        if (row_ok && j < n)
#pragma unroll
            for (int k = 0; k < M; k++)
                if (k < n) s += hr[k] * U_row(k, j);
        T[j] = s;
    }
    __syncthreads();
    if (on)
#pragma unroll
        for (int k = 0; k < M; k++) S.g[grp].rows[1][r][k] = T[k];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < M; j++) {        // C[r][j] = sum_k (T[r][k] g_k) T[j][k]
        double s = 0.0;
        if (row_ok && j < n)
#pragma unroll
            for (int k = 0; k < M; k++)
                if (k < n) s += (T[k] * S.g[grp].dg[k]) * S.g[grp].rows[1][j][k];
        A[j] = s;
    }
    __syncthreads();
    if (on)
#pragma unroll
        for (int k = 0; k < M; k++) S.g[grp].rows[0][r][k] = A[k];
    __syncthreads();
    // an eigensolve that hit the sweep cap fails its (walker, bin): NaN bigX entries
    // (so -lnL is NaN) and a sticky status bit (cmbl_status); the reference stops the run
    const unsigned long long gmask = ((1ull << M) - 1) << (on ? grp * M : 0);
    const bool failed = on && (__ballot(unconverged) & gmask) != 0;
    if (live && failed && r == 0) atomicOr(h.status, CMBL_STATUS_HL_NOCONV);
    // vecp = lower-triangle elements (MatrixToElements :917-931); bigX entries of this bin
    if (live) {
        double *x = xrows + (long long)w * h.Np + (long long)b * h.ncl_used;
        for (int u = r; u < h.ncl_used; u += M) {
            const int k = h.cl_use[u];
            int i = 0;
            while ((i + 1) * (i + 2) / 2 <= k) i++;
            const int j = k - i * (i + 1) / 2;
            x[u] = failed ? __builtin_nan("") : S.g[grp].rows[0][i][j];
        }
    }
#ifdef CMAMD_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    HL_STAMP(q9);
    if (lane == 0) {
        const unsigned long long q[10] = {q0, q1, q2, q3, q4, q5, q6, q7, q8, q9};
        for (int i = 0; i < 9; i++) atomicAdd(&g_hl_tp[i], q[i + 1] - q[i]);
        atomicAdd(&g_hl_tp[11], 1ull);
    }
#endif
}

// ------------------------------------------------------- exact (unbinned)
// like_approx = exact: per l, C = MapCl(l) + N_l (n x n over the used maps) and
// ExactChiSq (CMBlikes.f90:967-979)
//   chi2_l = (2l+1) fksy (tr M - n - ln det M),  M = C^-1/2 Chat_l C^-1/2.
// tr M = tr(C^-1 Chat) = |L^-1 R|_F^2 with C = L L^T and Chat = R R^T (R and
// ln det Chat = 2 sum ln R_ii from the host), and ln det M = ln det Chat - ln det C,
// so a thread needs one n x n Cholesky and a triangular solve instead of two
// eigendecompositions.  A C that is not positive definite gives NaN (the
// reference's C^-1/2 takes a negative eigenvalue to the power -1/2).
struct ExactDev {
    int n, ncl, lmin, lmax, bmin, nb, K;   // K: doubles per l row of tab
    int field[10], cmb[10];                // per element of the lower triangle (ElementsToMatrix order)
    const double *tab;                     // [nb][K]: N_l (ncl), R (ncl, lower packed), ln det Chat, (2l+1) fksy
    double aberration, log_cal_prior;
    int cal_index;
};
static constexpr int EXACT_MAXMAPS = 4;    // T, E, B, P
static constexpr int EXACT_WPB = 4;        // walkers per 256-thread block: one wave each

template <int N>
__global__ __launch_bounds__(256) void cmbl_exact_kernel(ExactDev x, const double *__restrict__ dl, long long ld_field,
                                                         long long ld_walker, const double *__restrict__ nuis,
                                                         long long ld_nuis, double *__restrict__ out, int W)
{
    constexpr int NC = N * (N + 1) / 2;
    const int lane = threadIdx.x & 63;
    const int w = blockIdx.x * EXACT_WPB + (threadIdx.x >> 6);
    if (w >= W) return;                                   // wave-uniform
    double calsq = 1.0;
    if (x.cal_index >= 0) {
        const double cal = nuis[(long long)w * ld_nuis + x.cal_index];
        calsq = cal * cal;
    }
    const double *Dw = dl + (long long)w * ld_walker;
    double acc = 0.0;
    for (int b = lane; b < x.nb; b += 64) {
        const int l = x.bmin + b;
        const double *t = x.tab + (long long)b * x.K;
        double C[NC];
#pragma unroll
        for (int e = 0; e < NC; e++) {                    // GetTheoryMapCls + AdaptTheoryForMaps :1022-1126
            const double *Df = Dw + (long long)x.field[e] * ld_field;
            double v = Df[l];
            if (x.aberration != 0.0 && x.cmb[e]) {        // AddAberration :1062-1101
                int la = l - 1, lb = l + 1;
                if (l == x.lmin) { la = l; lb = l + 2; }
                else if (l == x.lmax) { la = l - 2; lb = l; }
                const double ea = la, eb = lb, el = l;
                const double ca = Df[la] / (ea * (ea + 1)), cb = Df[lb] / (eb * (eb + 1));
                const double deriv = 0.5 * (cb - ca);
                v = v + x.aberration * (el * el * (el + 1) * deriv);
            }
            if (x.cal_index >= 0 && x.cmb[e]) v = v / calsq;
            C[e] = v + t[e];                              // C + NoiseM(bin) :1200-1202
        }
        // C = L L^T (lower packed, in place); ln det C
        double lndet_c = 0.0;
#pragma unroll
        for (int j = 0; j < N; j++) {
            double d = C[j * (j + 1) / 2 + j];
#pragma unroll
            for (int k = 0; k < j; k++) d -= C[j * (j + 1) / 2 + k] * C[j * (j + 1) / 2 + k];
            d = sqrt(d);                                  // NaN when C is not positive definite
            C[j * (j + 1) / 2 + j] = d;
            lndet_c += log(d);
#pragma unroll
            for (int i = j + 1; i < N; i++) {
                double s = C[i * (i + 1) / 2 + j];
#pragma unroll
                for (int k = 0; k < j; k++) s -= C[i * (i + 1) / 2 + k] * C[j * (j + 1) / 2 + k];
                C[i * (i + 1) / 2 + j] = s / d;
            }
        }
        // tr(C^-1 Chat) = |L^-1 R|_F^2, column by column of R (lower triangular)
        double tr = 0.0;
#pragma unroll
        for (int c = 0; c < N; c++) {
            double y[N];
#pragma unroll
            for (int i = 0; i < N; i++) {
                double s = (i >= c) ? t[x.ncl + i * (i + 1) / 2 + c] : 0.0;
#pragma unroll
                for (int k = 0; k < i; k++) s -= C[i * (i + 1) / 2 + k] * y[k];
                y[i] = s / C[i * (i + 1) / 2 + i];
                tr += y[i] * y[i];
            }
        }
        const double lndet_m = t[2 * x.ncl] - 2.0 * lndet_c;
        acc += t[2 * x.ncl + 1] * (tr - N - lndet_m);
    }
    // fixed-order wave reduction (deterministic)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    if (lane == 0) {
        double chisq = acc;
        if (x.log_cal_prior > 0 && x.cal_index >= 0) {   // :1222-1223
            const double lc = log(nuis[(long long)w * ld_nuis + x.cal_index]) / x.log_cal_prior;
            chisq = chisq + lc * lc;
        }
        out[w] = chisq / 2;
    }
}

// ------------------------------------------------------------------ host side

static std::vector<std::string> split_list(const std::string &s) { return split_ws(s); }

static int type_index(char ch) {   // TypeIndex: T E B P -> 1..4 (:134-144)
    const char *f = "TEBP";
    const char *p = std::strchr(f, ch);
    if (!p || !ch) fail(CMBL_ERR_FORMAT, "Invalid C_l part %c, must be one of: TEBP", ch);
    return (int)(p - f) + 1;
}

static std::string format_u(const std::string &fmt, int i) {   // FormatString(filename, i) for %u
    std::string s = fmt;
    size_t p = s.find("%u");
    if (p != std::string::npos) s.replace(p, 2, std::to_string(i));
    return s;
}

// File%LastTopComment (FileUtils.f90:1150-1168)
static std::string last_top_comment(const std::string &path) {
    std::ifstream f(path);
    if (!f) fail(CMBL_ERR_IO, "cannot read %s", path.c_str());
    std::string line, res;
    while (std::getline(f, line)) {
        size_t a = line.find_first_not_of(" \t\r");
        if (a == std::string::npos) continue;
        if (line[0] == '#') {
            std::string t = line.substr(1);
            size_t b = t.find_first_not_of(" \t");
            res = b == std::string::npos ? "" : t.substr(b);
            while (!res.empty() && (res.back() == ' ' || res.back() == '\r' || res.back() == '\t')) res.pop_back();
        } else {
            break;
        }
    }
    return res;
}

static double parse_double(const std::string &s) {
    std::string t = s;
    for (auto &ch : t)
        if (ch == 'd' || ch == 'D') ch = 'e';
    return std::stod(t);
}

static bool ini_logical(const Ini &ini, const std::string &key, bool def) {
    std::string v = ini.str(key);
    if (v.empty()) return def;
    const char ch = (char)std::toupper(v[0] == '.' && v.size() > 1 ? v[1] : v[0]);
    if (ch == 'T' || ch == '1' || ch == 'Y') return true;
    if (ch == 'F' || ch == '0' || ch == 'N') return false;
    fail(CMBL_ERR_FORMAT, "%s: bad logical %s = %s", ini.filename().c_str(), key.c_str(), v.c_str());
    return def;
}

static int ini_int(const Ini &ini, const std::string &key, bool required, int def) {
    std::string v = required ? ini.str_required(key) : ini.str(key);
    if (v.empty()) return def;
    return std::stoi(v);
}

static double ini_double(const Ini &ini, const std::string &key, double def) {
    std::string v = ini.str(key);
    return v.empty() ? def : parse_double(v);
}

struct Windows {                   // TBinWindows (:27-34) for bins bin_min..bin_max
    std::vector<int> in_i, in_j;   // required-map indices (1-based, i >= j; 0 = not required)
    std::vector<int> out;          // used cl index (1-based, 0 = not used)
    std::vector<double> W;         // [bin][win][L]
    std::vector<std::vector<double>> fix;   // per window: fixed spectrum over L (empty = theory)
    bool present = false;
};

struct CMBLikes final : Like {
    // ReadIni state
    bool has_map_names = false, bk = false, smica = false;
    std::vector<std::string> map_names, used_map_order;
    std::vector<int> map_fields, use_map, require_map, map_used_index, map_required_index, required_order;
    int approx = 0, nmaps = 0, nreq = 0, ncl = 0, ncl_used = 0, nsamp = 0;   // approx: 1 HL, 2 gaussian, 3 exact
    bool binned = true;
    double fksy = 1.0;                                              // fullsky_exact_fksy
    int lmin = 0, lmax = 0, nbins = 0, bin_min = 1, bin_max = 0, nb = 0;
    double aberration = 0.0, log_cal_prior = -1.0;
    int cal_index = -1;
    Windows bw, cw;
    std::vector<double> clhat, clnoise, clfid, fidcorr;   // [bin][ncl]
    std::vector<int> cl_use;                               // 0-based
    QuadForm qf;
    int nX = 0;
    // device tables
    CLDev dev{};
    HLDev hl{};
    DevBuf d_pairs, d_items, d_wts, d_wdir, d_sumoff, d_sumcols, d_sumconst, d_corroff, d_corrcols, d_corrconst,
        d_etox, d_fidcorr, d_noise, d_chat, d_cluse, d_bkmaps, d_bpnu, d_bpR, d_bpdnu, d_hlchat, d_hlcf, d_hlu0, d_hlv0;
    int max_field = 0, n_part_rows = 0;
    bool items_even = true, small_gauss = false;
    bool use_group = false;      // BK foregrounds: grouped-pair window kernel
    int n_gitem = 0;
    DevBuf d_gitems, d_gw, d_bplnu, d_logl80;
    int small_ntask = 0;
    SmallDev sdev{};
    DevBuf d_invcov, d_stasks, d_smt, d_sct;
    // window columns (one per bin and window entry with an output; main then
    // correction), the map pairs they read, and per element its columns; kept
    // so the work items can be rebuilt on other segment boundaries (window_resegment)
    struct HCol { int pair, lo, hi; const double *W; double cst; bool fixed; };
    std::vector<HCol> wcols;
    std::vector<CLPair> pairs;
    std::vector<std::vector<int>> w_emain, w_ecorr;
    std::vector<WItem> h_items;                     // direct-path work items (host copy)
    std::vector<std::vector<int>> h_item_cols;      // their columns (indices into wcols)
    std::map<int, std::vector<int>> seg_starts;     // theory field -> segment starts (relative l); default 256

    std::string cl_name(const std::vector<std::string> &names, int i, int j) const {   // Cl_i_j_name (:328-343)
        return has_map_names ? names[i - 1] + "x" + names[j - 1] : names[i - 1] + names[j - 1];
    }
    int map_index(const std::string &s) const {
        for (size_t k = 0; k < map_names.size(); k++)
            if (map_names[k] == s) return (int)k + 1;
        return -1;
    }
    void pair_to_map_indices(const std::string &S, int &i1, int &i2) const {   // :195-213
        if (S.size() == 2) {
            if (has_map_names) fail(CMBL_ERR_FORMAT, "CMBlikes: CL names must use MAP1xMAP2 names");
            i1 = map_index(S.substr(0, 1));
            i2 = map_index(S.substr(1, 1));
        } else {
            size_t ix = S.find('x');
            if (ix == std::string::npos) fail(CMBL_ERR_FORMAT, "CMBLikes: invalid spectrum name %s", S.c_str());
            i1 = map_index(S.substr(0, ix));
            i2 = map_index(S.substr(ix + 1));
        }
        if (i1 == -1 || i2 == -1) fail(CMBL_ERR_FORMAT, "CMBLikes: unrecognised map name %s", S.c_str());
    }
    // UseString_to_Cl_i_j (:262-281) with PairStringToUsedMapIndices (:215-231)
    void use_string_to_cl_i_j(const std::string &S, const std::vector<int> &used_index, std::vector<int> &ii,
                              std::vector<int> &jj) const {
        ii.clear();
        jj.clear();
        for (auto &t : split_list(S)) {
            int i1, i2;
            pair_to_map_indices(t, i1, i2);
            i1 = used_index[i1 - 1];
            i2 = used_index[i2 - 1];
            if (i2 > i1) std::swap(i1, i2);
            ii.push_back(i1);
            jj.push_back(i2);
        }
    }
    std::vector<int> use_string_to_cols(const std::string &S) const {   // :234-260
        std::vector<int> ii, jj, cols;
        use_string_to_cl_i_j(S, map_used_index, ii, jj);
        for (size_t k = 0; k < ii.size(); k++) {
            int ix = 0, c = 0;
            for (int a = 1; a <= nmaps; a++)
                for (int b = 1; b <= a; b++) {
                    ix++;
                    if (a == ii[k] && b == jj[k]) c = ix;
                }
            if (ii[k] == 0 || jj[k] == 0) c = 0;
            cols.push_back(c);
        }
        return cols;
    }
    int cols_from_order(const std::string &order, std::vector<int> &cols) const {   // GetColsFromOrder :345-369
        auto li = split_list(order);
        auto index_of = [&](const std::string &s) {
            for (size_t k = 0; k < li.size(); k++)
                if (li[k] == s) return (int)k + 1;
            return -1;
        };
        cols.assign(ncl, 0);
        int ix = 0;
        for (int i = 1; i <= nmaps; i++)
            for (int j = 1; j <= i; j++) {
                ix++;
                int i1 = index_of(cl_name(used_map_order, i, j));
                if (i1 == -1 && i != j) i1 = index_of(cl_name(used_map_order, j, i));
                if (i1 != -1) {
                    if (cols[ix - 1] > 0) fail(CMBL_ERR_FORMAT, "GetColsFromOrder: duplicate CL type");
                    cols[ix - 1] = i1;
                }
            }
        return (int)li.size();
    }
    // ReadClArr (:146-193): Cl [bin_min..bin_max][ncl]
    bool read_cl_arr(const Ini &ini, const std::string &base, std::vector<double> &cl, bool optional) const {
        std::string fn = ini.relative_filename(base + "_file", !optional);
        if (fn.empty()) return false;
        std::string order = ini.str(base + "_order"), incols;
        if (order.empty()) {
            incols = last_top_comment(fn);
            if (incols.empty()) fail(CMBL_ERR_FORMAT, "No column order given for %s", fn.c_str());
        } else {
            incols = "L " + order;
        }
        std::vector<int> cols;
        const int norder = cols_from_order(incols, cols) - 1;
        cl.assign((size_t)nb * ncl, 0.0);
        auto rows = load_txt(fn);
        int ll = -1;
        for (auto &r : rows) {
            if ((int)r.size() < 1 + norder) fail(CMBL_ERR_FORMAT, "CMBLikes_ReadClArr: error reading line %s", fn.c_str());
            const int l = (int)r[0];
            ll = l;
            if (l >= bin_min && l <= bin_max)
                for (int ix = 0; ix < ncl; ix++)
                    if (cols[ix] != 0) cl[(size_t)(l - bin_min) * ncl + ix] = r[cols[ix] - 1];
        }
        if (ll < bin_max) fail(CMBL_ERR_FORMAT, "CMBLikes_ReadClArr: C_l file does not go up to maximum used: %d (%s)",
                               bin_max, fn.c_str());
        return true;
    }
    void read_bin_windows(const Ini &ini, const std::string &type, Windows &bwin) {   // ReadBinWindows :371-464
        const int L = lmax - lmin + 1;
        std::string fname = ini.str_required(type + "_files");
        std::string order1 = ini.str_required(type + "_in_order");
        std::string order2 = ini.str(type + "_out_order", order1);
        if (order2.empty()) order2 = order1;
        use_string_to_cl_i_j(order1, map_required_index, bwin.in_i, bwin.in_j);
        bwin.out = use_string_to_cols(order2);
        const int norder = (int)bwin.in_i.size();
        if (norder != (int)bwin.out.size())
            fail(CMBL_ERR_FORMAT, "%s_in_order and %s_out_order must have same number of CL", type.c_str(), type.c_str());
        bwin.W.assign((size_t)nb * norder * L, 0.0);
        for (int b = bin_min; b <= bin_max; b++) {
            std::string S = ini.resolve_path(format_u(fname, b));
            auto rows = load_txt(S);
            for (auto &r : rows) {
                if ((int)r.size() < 1 + norder) fail(CMBL_ERR_FORMAT, "ReadBinWindows: error reading line %s", S.c_str());
                const int l = (int)r[0];
                if (l >= lmin && l <= lmax)
                    for (int k = 0; k < norder; k++) bwin.W[((size_t)(b - bin_min) * norder + k) * L + (l - lmin)] = r[1 + k];
            }
        }
        bwin.fix.assign(norder, {});
        std::string fixf = ini.relative_filename(type + "_fix_cl_file", false);
        if (!fixf.empty()) {
            std::string o1 = ini.str(type + "_fix_cl_file_order");
            if (o1.empty()) {
                o1 = last_top_comment(fixf);
                if (o1.empty()) fail(CMBL_ERR_FORMAT, "No column order given for %s", fixf.c_str());
                while (!o1.empty() && (o1[0] == ' ' || o1[0] == 'L')) o1 = o1.substr(1);
            }
            std::vector<int> fi, fj, ui, uj;
            use_string_to_cl_i_j(o1, map_required_index, fi, fj);
            use_string_to_cl_i_j(ini.str_required(type + "_fix_cl"), map_required_index, ui, uj);
            auto rows = load_txt(fixf);
            for (size_t u = 0; u < ui.size(); u++) {
                if (ui[u] == 0 || uj[u] == 0) continue;
                int idx = -1;
                for (size_t k = 0; k < fi.size(); k++)
                    if (fi[k] == ui[u] && fj[k] == uj[u]) { idx = (int)k; break; }
                if (idx < 0) fail(CMBL_ERR_FORMAT, "ReadBinWindows: fix_cl uses CL not in the fix_cl_file");
                std::vector<double> spec(L, 0.0);
                for (auto &r : rows) {
                    const int l = (int)r[0];
                    if (l >= lmin && l <= lmax && (int)r.size() > idx + 1) spec[l - lmin] = r[idx + 1];
                }
                for (int k = 0; k < norder; k++)
                    if (bwin.in_i[k] == ui[u] && bwin.in_j[k] == uj[u]) bwin.fix[k] = spec;
            }
        }
        bwin.present = true;
    }

    CMBLikes(const Ini &ini, const std::string &tag_) {
        tag = tag_;
        bk = (tag == "BKPLANCK");
        smica = (tag == "SMICA");       // TSmica_planck (CMB.f90:94-95)
        name = ini.str("name");
        if (name.empty()) {
            std::string fn = ini.filename();
            size_t s = fn.find_last_of('/');
            fn = fn.substr(s == std::string::npos ? 0 : s + 1);
            size_t d = fn.find_last_of('.');
            name = d == std::string::npos ? fn : fn.substr(0, d);
        }
        // ---- CMBLikes_ReadIni (:466-749)
        std::string fmt = ini.str("dataset_format");
        if (fmt == "CMBLike") fail(CMBL_ERR_FORMAT, "CMBLikes dataset_format now CMBLike2");
        if (!fmt.empty() && fmt != "CMBLike2") fail(CMBL_ERR_FORMAT, "CMBLikes wrong dataset_format");
        std::string S = ini.str("map_names");
        has_map_names = !S.empty();
        if (has_map_names) {
            map_names = split_list(S);
            auto mf = split_list(ini.str_required("map_fields"));
            if (mf.size() != map_names.size()) fail(CMBL_ERR_FORMAT, "CMBLikes: number of map_fields does not match map_names");
            for (auto &f : mf) map_fields.push_back(type_index(f[0]));
        } else {
            map_names = {"T", "E", "B", "P"};
            map_fields = {1, 2, 3, 4};
        }
        bool use_field[5] = {false, false, false, false, false};
        S = ini.str("fields_use");
        if (!S.empty()) {
            for (auto &f : split_list(S)) use_field[type_index(f[0])] = true;
        } else {
            if (!has_map_names) fail(CMBL_ERR_FORMAT, "CMBlikes: must have fields_use or map_names");
            for (int i = 1; i <= 4; i++) use_field[i] = true;
        }
        const int nm = (int)map_names.size();
        use_map.assign(nm, 0);
        S = ini.str("maps_use");
        if (!S.empty()) {
            for (auto &m : split_list(S)) {
                const int j = map_index(m);
                if (j == -1) fail(CMBL_ERR_FORMAT, "CMBlikes: maps_use item not found - %s", m.c_str());
                use_map[j - 1] = 1;
            }
        } else {
            for (int i = 0; i < nm; i++) use_map[i] = use_field[map_fields[i]];
        }
        require_map = use_map;
        if (has_map_names) {
            S = ini.str("maps_required");
            if (ini.has("fields_required")) fail(CMBL_ERR_FORMAT, "CMBLikes: use maps_required not fields_required");
        } else {
            S = ini.str("fields_required");
        }
        for (auto &m : split_list(S)) {
            const int j = map_index(m);
            if (j == -1) fail(CMBL_ERR_FORMAT, "CMBlikes: required item not found - %s", m.c_str());
            require_map[j - 1] = 1;
        }
        bool req_field[5] = {false, false, false, false, false};
        for (int i = 0; i < nm; i++)
            if (require_map[i]) req_field[map_fields[i]] = true;
        std::string la = ini.str_required("like_approx");
        if (la == "HL") approx = 1;
        else if (la == "gaussian") approx = 2;
        else if (la == "exact") approx = 3;
        else fail(CMBL_ERR_FORMAT, "CMBlikes: unknown like_approx %s", la.c_str());
        for (int i = 0; i < nm; i++) {
            nmaps += use_map[i];
            nreq += require_map[i];
        }
        if (nmaps < 1) fail(CMBL_ERR_FORMAT, "CMBlikes: no maps used");
        if (approx == 1 && nmaps > CL_MAXMAPS) fail(CMBL_ERR_UNSUPPORTED, "CMBlikes HL: at most %d maps", CL_MAXMAPS);
        if (approx == 3 && nmaps > EXACT_MAXMAPS)
            fail(CMBL_ERR_UNSUPPORTED, "CMBlikes exact: at most %d maps", EXACT_MAXMAPS);
        if (approx == 3 && bk) fail(CMBL_ERR_UNSUPPORTED, "BKPLANCK with like_approx = exact is not supported");
        if (approx == 3 && smica) fail(CMBL_ERR_UNSUPPORTED, "SMICA with like_approx = exact is not supported");
        if (nreq > CL_MAXREQ) fail(CMBL_ERR_UNSUPPORTED, "CMBlikes: at most %d required maps", CL_MAXREQ);
        map_required_index.assign(nm, 0);
        map_used_index.assign(nm, 0);
        int ix = 0;
        for (int i = 0; i < nm; i++)
            if (require_map[i]) {
                map_required_index[i] = ++ix;
                required_order.push_back(i + 1);
            }
        ix = 0;
        for (int i = 0; i < nm; i++)
            if (use_map[i]) {
                map_used_index[i] = ++ix;
                used_map_order.push_back(map_names[i]);
            }
        ncl = nmaps * (nmaps + 1) / 2;
        lmin = ini_int(ini, "cl_lmin", true, 0);
        lmax = ini_int(ini, "cl_lmax", true, 0);
        if (!ini.has("binned")) fail(CMBL_ERR_FORMAT, "CMBlikes: binned not given");   // Read_Logical('binned') :597
        binned = ini_logical(ini, "binned", false);
        aberration = ini_double(ini, "aberration_coeff", 0.0);
        if (binned) {
            if (approx == 3) fail(CMBL_ERR_FORMAT, "CMBLikes: exact like cannot be binned!");   // :1185
            nbins = ini_int(ini, "nbins", false, 0);
            bin_min = ini_int(ini, "use_min", false, 1);
            bin_max = ini_int(ini, "use_max", false, nbins);
            if (bin_min < 1 || bin_min > nbins || bin_max < bin_min || bin_max > nbins)
                fail(CMBL_ERR_FORMAT, "CMBlikes: use_min/use_max outside 1..nbins");
        } else {
            // unbinned (:601-605, :636-637): one "bin" per l; only the exact
            // likelihood (the reference marks unbinned HL / gaussian untested)
            if (approx != 3)
                fail(CMBL_ERR_UNSUPPORTED, "CMBlikes: unbinned HL / gaussian likelihoods are not supported "
                                           "(untested in the reference)");
            if (nmaps != nreq) fail(CMBL_ERR_FORMAT, "CMBlikes: Unbinned must have required==used");   // :1188
            nbins = lmax - lmin + 1;
            bin_min = ini_int(ini, "use_min", false, lmin);
            bin_max = ini_int(ini, "use_max", false, lmax);
            if (bin_min < lmin || bin_min > lmax || bin_max < bin_min || bin_max > lmax)
                fail(CMBL_ERR_FORMAT, "CMBlikes: use_min/use_max outside cl_lmin..cl_lmax");
            if (lmax - lmin < 2 && aberration != 0.0)
                fail(CMBL_ERR_FORMAT, "CMBlikes: aberration needs cl_lmax >= cl_lmin + 2");
        }
        nb = bin_max - bin_min + 1;
        if (binned) read_bin_windows(ini, "bin_window", bw);
        read_cl_arr(ini, "cl_hat", clhat, false);
        if (approx == 1) read_cl_arr(ini, "cl_fiducial", clfid, false);
        if (approx == 3) fksy = ini_double(ini, "fullsky_exact_fksy", 1.0);      // :645-648
        const bool includes_noise = ini_logical(ini, "cl_hat_includes_noise", false);
        bool have_noise = false;
        if (approx != 2 || includes_noise) {
            read_cl_arr(ini, "cl_noise", clnoise, false);
            have_noise = true;
            if (!includes_noise) {
                for (size_t k = 0; k < clhat.size(); k++) clhat[k] = clhat[k] + clnoise[k];
            } else if (approx == 2) {
                for (size_t k = 0; k < clhat.size(); k++) clhat[k] = clhat[k] - clnoise[k];
                have_noise = false;
            }
        }
        for (int i = 1; i <= 4; i++)
            if (req_field[i]) cl_lmax[(i - 1) * 4 + (i - 1)] = lmax;
        if (req_field[1] && req_field[2]) cl_lmax[(2 - 1) * 4 + (1 - 1)] = lmax;
        if (ini.has("point_source_cl") || ini.has("beam_modes_file"))
            fail(CMBL_ERR_FORMAT, "dataset uses keywords no longer supported");
        bool fid_incl_noise = false;
        if (approx != 2) fid_incl_noise = ini_logical(ini, "cl_fiducial_includes_noise", false);
        // per-bin matrices (:711-724)
        std::vector<double> chatM((size_t)nb * nmaps * nmaps), cfh((size_t)nb * nmaps * nmaps);
        auto to_matrix = [&](const double *X, double *M) {
            int q = 0;
            for (int i = 0; i < nmaps; i++)
                for (int j = 0; j <= i; j++, q++) M[i * nmaps + j] = M[j * nmaps + i] = X[q];
        };
        for (int b = 0; b < nb; b++) {
            to_matrix(&clhat[(size_t)b * ncl], &chatM[(size_t)b * nmaps * nmaps]);
            if (approx == 1) {
                std::vector<double> f(clfid.begin() + (size_t)b * ncl, clfid.begin() + (size_t)(b + 1) * ncl);
                if (!fid_incl_noise)
                    for (int k = 0; k < ncl; k++) f[k] = f[k] + clnoise[(size_t)b * ncl + k];
                std::vector<double> M((size_t)nmaps * nmaps);
                to_matrix(f.data(), M.data());
                sym_power(M, nmaps, 0.5);
                std::copy(M.begin(), M.end(), cfh.begin() + (size_t)b * nmaps * nmaps);
            }
        }
        if (approx != 3) read_covmat(ini);        // :726-728
        std::vector<double> fc;
        if (!binned && ini.has("linear_correction_fiducial_file"))
            fail(CMBL_ERR_UNSUPPORTED, "CMBlikes: linear corrections of an unbinned likelihood are not supported");
        if (read_cl_arr(ini, "linear_correction_fiducial", fc, true)) {
            fidcorr = fc;
            read_bin_windows(ini, "linear_correction_bin_window", cw);
        }
        std::string cp = ini.relative_filename("calibration_param", false);
        if (!cp.empty()) {
            nuisance_names = load_paramnames(cp, &n_nuis, &derived_names, &n_derived);
            cal_index = n_nuis - 1;
            log_cal_prior = ini_double(ini, "log_calibration_prior", -1.0);
        }
        // ---- Tsmica_planck_ReadIni (CMBlikes.f90:1281-1293): after the base ReadIni
        // (which may have set a calibration index from calibration_param), the
        // nuisance names are replaced by nuisance_params (loadParamNames ->
        // nuisance_params%init), and calibration_paramname, when given, sets the
        // calibration index to that name's position in them (ParamNames%Index:
        // -1, i.e. no calibration, for an unknown name)
        if (smica) {
            nuisance_names = load_paramnames(ini.relative_filename("nuisance_params", true), &n_nuis, &derived_names,
                                             &n_derived);
            if (n_nuis < 5) fail(CMBL_ERR_FORMAT, "SMICA: nuisance_params needs the foreground parameters A1 n1 n1run A2 n2");
            if (ini.has("calibration_paramname")) {
                const std::string cn = ini.str("calibration_paramname");
                const auto nm = split_ws(nuisance_names), dn = split_ws(derived_names);
                int ix = -1;
                for (size_t k = 0; k < nm.size() && ix < 0; k++)
                    if (nm[k] == cn) ix = (int)k;
                for (size_t k = 0; k < dn.size() && ix < 0; k++)
                    if (dn[k] == cn) fail(CMBL_ERR_FORMAT, "SMICA: calibration_paramname %s is a derived parameter", cn.c_str());
                cal_index = ix;   // -1: none
            }
        }
        // ---- TBK_planck_ReadIni (CMB_BK_Planck.f90:36-70).  As for SMICA, a
        // calibration_param read by the base ReadIni (:43) sets the calibration index
        // to its name count and loadParamNames (:46, nuisance_params%init) then replaces
        // the names: the index stays and points into the BK parameters
        std::vector<BKMap> bkm;
        std::vector<double> bnu, bR, bdnu;
        if (bk) {
            nuisance_names = load_paramnames(ini.relative_filename("nuisance_params", true), &n_nuis);
            if (n_nuis < BK_NPARAM) fail(CMBL_ERR_FORMAT, "BKPLANCK: nuisance_params needs %d parameters", BK_NPARAM);
            dev.fpivot_dust = ini_double(ini, "fpivot_dust", 353.0);
            dev.fpivot_sync = ini_double(ini, "fpivot_sync", 23.0);
            dev.decorr_dust[0] = ini_double(ini, "fpivot_dust_decorr(1)", 217.0);
            dev.decorr_dust[1] = ini_double(ini, "fpivot_dust_decorr(2)", 353.0);
            dev.decorr_sync[0] = ini_double(ini, "fpivot_sync_decorr(1)", 23.0);
            dev.decorr_sync[1] = ini_double(ini, "fpivot_sync_decorr(2)", 33.0);
            auto lform = [&](const std::string &k) {
                std::string v = ini.str(k, "flat");
                return v == "lin" ? 1 : v == "quad" ? 2 : 0;
            };
            dev.lform_dust = lform("lform_dust_decorr");
            dev.lform_sync = lform("lform_sync_decorr");
            // the reference reads nmaps_required bandpasses named by used_map_order (:64-66),
            // which holds only the nmaps used maps: a required map beyond them has no defined
            // bandpass there, so the case is refused rather than given a meaning
            if (nreq != nmaps) fail(CMBL_ERR_UNSUPPORTED, "BKPLANCK: maps_required beyond maps_use not supported");
            const double G = ghz_kelvin();
            for (int i = 0; i < nreq; i++) {
                const std::string &mn = used_map_order[i];
                auto R = load_txt(ini.relative_filename("bandpass[" + mn + "]", true));
                const int n = (int)R.size();
                if (n < 2) fail(CMBL_ERR_FORMAT, "bandpass for %s too short", mn.c_str());
                BKMap m{};
                m.off = (int)bnu.size();
                m.n = n;
                std::vector<double> dnu(n);
                dnu[0] = R[1][0] - R[0][0];
                for (int k = 1; k < n - 1; k++) dnu[k] = (R[k + 1][0] - R[k - 1][0]) / 2;
                dnu[n - 1] = R[n - 1][0] - R[n - 2][0];
                double th_int = 0, s1 = 0, s2 = 0;
                for (int k = 0; k < n; k++) {
                    const double nu = R[k][0], r = R[k][1];
                    const double e = std::exp(G * nu / BK_TCMB);
                    th_int += dnu[k] * r * (nu * nu * nu * nu) * e / ((e - 1) * (e - 1));
                    s1 += dnu[k] * nu * r;
                    s2 += dnu[k] * r;
                    bnu.push_back(nu);
                    bR.push_back(r);
                    bdnu.push_back(dnu[k]);
                }
                auto th0 = [&](double nu0) {
                    const double e = std::exp(G * nu0 / BK_TCMB);
                    return (nu0 * nu0 * nu0 * nu0) * e / ((e - 1) * (e - 1));
                };
                m.th_dust = th_int / th0(dev.fpivot_dust);
                m.th_sync = th_int / th0(dev.fpivot_sync);
                m.nu_bar = s1 / s2;
                m.bc = mn.find("95") != std::string::npos ? 1 : mn.find("150") != std::string::npos ? 2
                       : mn.find("220") != std::string::npos ? 3 : 0;
                bkm.push_back(m);
            }
        }
        if (approx == 3) build_exact(chatM);
        else build_device(have_noise, chatM, cfh, bkm, bnu, bR, bdnu);
    }

    // like_approx = exact: per-l table [nb][K] = N_l (ncl) | chol(Chat_l) (ncl) | ln det Chat_l | (2l+1) fksy
    ExactDev xdev{};
    DevBuf d_xtab;
    void build_exact(const std::vector<double> &chatM) {
        xdev.n = nmaps;
        xdev.ncl = ncl;
        xdev.lmin = lmin;
        xdev.lmax = lmax;
        xdev.bmin = bin_min;
        xdev.nb = nb;
        xdev.K = 2 * ncl + 2;
        std::vector<double> tab((size_t)nb * xdev.K, 0.0);
        for (int b = 0; b < nb; b++) {
            double *t = &tab[(size_t)b * xdev.K];
            for (int e = 0; e < ncl; e++) t[e] = clnoise[(size_t)b * ncl + e];
            // Chat = R R^T (Matrix_Cholesky, as MatrixSym_LogDet :619-634 does for M)
            const double *M = &chatM[(size_t)b * nmaps * nmaps];
            std::vector<double> R((size_t)nmaps * nmaps, 0.0);
            double lndet = 0.0;
            for (int j = 0; j < nmaps; j++) {
                double d = M[j * nmaps + j];
                for (int k = 0; k < j; k++) d -= R[j * nmaps + k] * R[j * nmaps + k];
                if (!(d > 0)) fail(CMBL_ERR_NUMERIC, "CMBlikes exact: cl_hat at l = %d is not positive definite", bin_min + b);
                d = std::sqrt(d);
                R[j * nmaps + j] = d;
                lndet += std::log(d);
                for (int i = j + 1; i < nmaps; i++) {
                    double v = M[i * nmaps + j];
                    for (int k = 0; k < j; k++) v -= R[i * nmaps + k] * R[j * nmaps + k];
                    R[i * nmaps + j] = v / d;
                }
            }
            for (int i = 0, q = 0; i < nmaps; i++)
                for (int j = 0; j <= i; j++, q++) t[ncl + q] = R[i * nmaps + j];
            t[2 * ncl] = 2.0 * lndet;
            t[2 * ncl + 1] = (2.0 * (bin_min + b) + 1.0) * fksy;
        }
        // element (i, j), i >= j, of the lower triangle -> theory field (MapPair_to_Theory_i_j :284-299)
        for (int i = 1, q = 0; i <= nmaps; i++)
            for (int j = 1; j <= i; j++, q++) {
                int f1 = map_fields[required_order[i - 1] - 1], f2 = map_fields[required_order[j - 1] - 1];
                if (f2 > f1) std::swap(f1, f2);
                xdev.field[q] = f1 * (f1 - 1) / 2 + (f2 - 1);
                xdev.cmb[q] = (f1 <= 3 && f2 <= 3);
                max_field = std::max(max_field, xdev.field[q]);
            }
        d_xtab.alloc(tab.size() * 8);
        d_xtab.upload(tab.data(), tab.size() * 8);
        xdev.tab = d_xtab.as<double>();
        xdev.aberration = aberration;
        xdev.cal_index = cal_index;
        xdev.log_cal_prior = log_cal_prior;
    }

    std::vector<double> invcov;
    void read_covmat(const Ini &ini) {   // ReadCovmat (:752-859), binned
        std::string covmat_cl = ini.str_required("covmat_cl");
        std::string fn = ini.relative_filename("covmat_fiducial", true);
        const double scale = ini_double(ini, "covmat_scale", 1.0);
        auto cl_in = use_string_to_cols(covmat_cl);
        const int num_in = (int)cl_in.size();
        std::vector<int> cov_cl_used;
        for (int i = 0; i < num_in; i++)
            if (cl_in[i] != 0) {
                cl_use.push_back(cl_in[i] - 1);
                cov_cl_used.push_back(i);
            }
        ncl_used = (int)cl_use.size();
        if (ncl_used == 0) fail(CMBL_ERR_FORMAT, "CMBlikes: covmat_cl selects no used spectra");
        const int nin = num_in * nbins;
        std::vector<double> cov;
        for (auto &r : load_txt(fn)) cov.insert(cov.end(), r.begin(), r.end());
        if ((long long)cov.size() < (long long)nin * nin)
            fail(CMBL_ERR_FORMAT, "%s: covariance needs %d x %d entries", fn.c_str(), nin, nin);
        nX = nb * ncl_used;
        invcov.assign((size_t)nX * nX, 0.0);
        for (int bx = bin_min; bx <= bin_max; bx++)
            for (int by = bin_min; by <= bin_max; by++)
                for (int a = 0; a < ncl_used; a++)
                    for (int b = 0; b < ncl_used; b++)
                        invcov[(size_t)((bx - bin_min) * ncl_used + a) * nX + (by - bin_min) * ncl_used + b] =
                            scale * cov[(size_t)((bx - 1) * num_in + cov_cl_used[a]) * nin + (by - 1) * num_in +
                                        cov_cl_used[b]];
        spd_inverse(invcov, nX);
    }

    // Work items of the window stage, their partial rows, and the per-element
    // row lists and small-gaussian tasks that consume them (re-run by
    // window_resegment; the results depend on the segment boundaries only
    // through the summation split of each window's dot product).
    void build_items() {
        const int L = lmax - lmin + 1;
        const int nE = nb * ncl;
        auto &cols = wcols;
        max_field = 0;
        // work items: per pair, per l chunk, the overlapping columns in groups of WK_COLS
        std::vector<WItem> items;
        std::vector<double> wdense, wdirect;
        std::vector<std::vector<int>> col_parts(cols.size());
        int nrows = 0;
        const int SEG = WK_CHUNK * WK_NCH;
        // BK foregrounds without aberration: grouped-pair items (cmbl_window_group),
        // when no pair has more than 16 window columns
        use_group = bk && aberration == 0.0;
        if (use_group) {
            std::vector<int> per_pair(pairs.size(), 0);
            for (auto &cc : cols)
                if (!cc.fixed && ++per_pair[cc.pair] > 16) use_group = false;
        }
        std::vector<GItem> gitems;
        std::vector<double> gw;
        if (use_group) {
            std::map<int, std::vector<int>> by_field;
            for (size_t p = 0; p < pairs.size(); p++) by_field[pairs[p].field].push_back((int)p);
            for (auto &fv : by_field)
                for (size_t g0 = 0; g0 < fv.second.size(); g0 += GP) {
                    const int npair = (int)std::min<size_t>(GP, fv.second.size() - g0);
                    for (int sg = 0; sg < (L + GSEG - 1) / GSEG; sg++) {
                        const int c0 = sg * GSEG, c1 = std::min(L - 1, c0 + GSEG - 1);
                        std::vector<std::vector<int>> sel(npair);
                        int lo = c1 + 1, hi = c0 - 1;
                        for (int g = 0; g < npair; g++)
                            for (size_t ci = 0; ci < cols.size(); ci++)
                                if (!cols[ci].fixed && cols[ci].pair == fv.second[g0 + g] && cols[ci].hi >= c0 &&
                                    cols[ci].lo <= c1) {
                                    sel[g].push_back((int)ci);
                                    lo = std::min(lo, std::max(c0, cols[ci].lo));
                                    hi = std::max(hi, std::min(c1, cols[ci].hi));
                                }
                        if (hi < lo) continue;
                        GItem it{};
                        it.field = fv.first;
                        it.npair = npair;
                        it.l0 = (lo + lmin) & ~1;      // even: 16-byte loads (>= lmin - 1; profiles are 0 there)
                        it.nstep = (hi + lmin - it.l0 + 32) / 32;
                        it.woff = (long long)gw.size();
                        const int Lp = it.nstep * 32;
                        for (int g = 0; g < GP; g++) {
                            it.pair[g] = g < npair ? fv.second[g0 + g] : 0;
                            it.ncol[g] = g < npair ? (int)sel[g].size() : 0;
                            it.part[g] = nrows;
                            for (int cc = 0; cc < 16; cc++)
                                for (int l = 0; l < Lp; l++) {
                                    const int jl = it.l0 + l - lmin;
                                    gw.push_back(g < npair && cc < it.ncol[g] && jl >= lo && jl <= hi
                                                     ? cols[sel[g][cc]].W[jl] : 0.0);
                                }
                            if (g < npair)
                                for (int ci : sel[g]) col_parts[ci].push_back(nrows++);
                        }
                        gitems.push_back(it);
                    }
                }
            for (auto &p : pairs) max_field = std::max(max_field, p.field);
        }
        n_gitem = (int)gitems.size();
        d_gitems.alloc(std::max<size_t>(16, gitems.size() * sizeof(GItem)));
        if (!gitems.empty()) d_gitems.upload(gitems.data(), gitems.size() * sizeof(GItem));
        d_gw.alloc(std::max<size_t>(16, gw.size() * 8));
        if (!gw.empty()) d_gw.upload(gw.data(), gw.size() * 8);
        h_items.clear();
        h_item_cols.clear();
        for (size_t p = 0; p < (use_group ? 0 : pairs.size()); p++) {
            std::vector<int> segs;
            auto fs = seg_starts.find(pairs[p].field);
            if (fs != seg_starts.end()) segs = fs->second;
            else
                for (int c = 0; c < L; c += SEG) segs.push_back(c);
            for (size_t sg = 0; sg < segs.size(); sg++) {
                const int c0 = segs[sg], c1 = std::min(L - 1, sg + 1 < segs.size() ? segs[sg + 1] - 1 : L - 1);
                if (c1 < c0) continue;
                std::vector<int> sel;
                for (size_t ci = 0; ci < cols.size(); ci++)
                    if (!cols[ci].fixed && cols[ci].pair == (int)p && cols[ci].hi >= c0 && cols[ci].lo <= c1)
                        sel.push_back((int)ci);
                for (size_t g0 = 0; g0 < sel.size(); g0 += WK_COLS) {
                    const size_t g1 = std::min(sel.size(), g0 + WK_COLS);
                    int lo = c1, hi = c0;
                    for (size_t g = g0; g < g1; g++) {
                        lo = std::min(lo, std::max(c0, cols[sel[g]].lo));
                        hi = std::max(hi, std::min(c1, cols[sel[g]].hi));
                    }
                    if ((lo + lmin) % 2 == 1 && lo > c0) lo--;     // even l0: 16-byte theory loads
                    WItem it{};
                    it.pair = (int)p;
                    it.l0 = lo + lmin;
                    it.l1 = hi + lmin;
                    it.ncol = (int)(g1 - g0);
                    it.part = nrows;
                    it.nch = (hi - lo + WK_CHUNK) / WK_CHUNK;
                    it.woff = (long long)wdense.size();
                    for (int l = lo; l < lo + it.nch * WK_CHUNK; l++)   // [nch][WK_CHUNK][WK_COLS], zero padded
                        for (int g = 0; g < WK_COLS; g++)
                            wdense.push_back(l <= hi && g0 + g < g1 ? cols[sel[g0 + g]].W[l] : 0.0);
                    it.woff2 = (long long)wdirect.size();
                    const int ncb = (it.ncol + 15) / 16;
                    for (int ch = 0; ch < it.nch; ch++)         // [nch][ncb][16][WK_CHUNK], zero padded
                        for (int cb = 0; cb < ncb; cb++)
                            for (int g = 16 * cb; g < 16 * cb + 16; g++)
                                for (int k = 0; k < WK_CHUNK; k++) {
                                    const int l = lo + ch * WK_CHUNK + k;
                                    wdirect.push_back(l <= hi && g0 + g < g1 ? cols[sel[g0 + g]].W[l] : 0.0);
                                }
                    for (size_t g = g0; g < g1; g++) col_parts[sel[g]].push_back(nrows++);
                    items.push_back(it);
                    h_item_cols.emplace_back(sel.begin() + g0, sel.begin() + g1);
                }
            }
        }
        h_items = items;
        n_part_rows = nrows;
        items_even = true;
        for (auto &it : items) items_even = items_even && (it.l0 % 2 == 0);
        for (auto &it : items) max_field = std::max(max_field, pairs[it.pair].field);
        // per element: the partial rows of its columns in window order, and the fixed-spectrum constants
        auto flatten = [&](const std::vector<std::vector<int>> &lists, std::vector<int> &off, std::vector<int> &rows,
                           std::vector<double> &cst) {
            off.assign(lists.size() + 1, 0);
            cst.assign(lists.size(), 0.0);
            for (size_t e = 0; e < lists.size(); e++) {
                off[e] = (int)rows.size();
                for (int ci : lists[e]) {
                    rows.insert(rows.end(), col_parts[ci].begin(), col_parts[ci].end());
                    cst[e] += cols[ci].cst;
                }
            }
            off[lists.size()] = (int)rows.size();
        };
        std::vector<int> main_off, main_rows, corr_off, corr_rows;
        std::vector<double> main_cst, corr_cst;
        flatten(w_emain, main_off, main_rows, main_cst);
        flatten(w_ecorr, corr_off, corr_rows, corr_cst);
        {   // small-gaussian tasks: each element's rows in runs of <= 8 (main rows, then corr rows)
            std::vector<SmallTask> tasks;
            std::vector<int> rows_all(main_rows);
            rows_all.insert(rows_all.end(), corr_rows.begin(), corr_rows.end());
            std::vector<int> mt(nE + 1), ct(nE + 1);
            for (int e = 0; e < nE; e++) {
                mt[e] = (int)tasks.size();
                for (int q = main_off[e]; q < main_off[e + 1]; q += 8)
                    tasks.push_back({q, std::min(8, main_off[e + 1] - q)});
            }
            mt[nE] = (int)tasks.size();
            const int base = (int)main_rows.size();
            for (int e = 0; e < nE; e++) {
                ct[e] = (int)tasks.size();
                for (int q = corr_off[e]; q < corr_off[e + 1]; q += 8)
                    tasks.push_back({base + q, std::min(8, corr_off[e + 1] - q)});
            }
            ct[nE] = (int)tasks.size();
            small_ntask = (int)tasks.size();
            auto up2 = [](DevBuf &d, const void *p, size_t bytes) {
                d.alloc(std::max<size_t>(bytes, 16));
                if (bytes) d.upload(p, bytes);
            };
            std::vector<int> trow(tasks.size() * 8, -1);
            for (size_t t = 0; t < tasks.size(); t++)
                for (int u = 0; u < tasks[t].count; u++) trow[8 * t + u] = rows_all[tasks[t].first + u];
            up2(d_stasks, trow.data(), trow.size() * 4);
            up2(d_smt, mt.data(), mt.size() * 4);
            up2(d_sct, ct.data(), ct.size() * 4);
        }
        auto up = [](DevBuf &d, const void *p, size_t bytes) {
            d.alloc(std::max<size_t>(bytes, 16));
            if (bytes) d.upload(p, bytes);
        };
        up(d_items, items.data(), items.size() * sizeof(WItem));
        up(d_wts, wdense.data(), wdense.size() * 8);
        up(d_wdir, wdirect.data(), wdirect.size() * 8);
        up(d_sumoff, main_off.data(), main_off.size() * 4);
        up(d_sumcols, main_rows.data(), main_rows.size() * 4);
        up(d_sumconst, main_cst.data(), main_cst.size() * 8);
        up(d_corroff, corr_off.data(), corr_off.size() * 4);
        up(d_corrcols, corr_rows.data(), corr_rows.size() * 4);
        up(d_corrconst, corr_cst.data(), corr_cst.size() * 8);
        small_gauss = approx == 2 && nX <= SMALL_NX && small_ntask <= SMALL_MAXTASK;
        sdev.ntask = small_ntask;
        sdev.trow = d_stasks.as<int>();
        sdev.e_main_t = d_smt.as<int>();
        sdev.e_corr_t = d_sct.as<int>();
        dev.nitem = (int)items.size();
        dev.items = d_items.as<WItem>();
        dev.wdense = d_wts.as<double>();
        dev.wdirect = d_wdir.as<double>();
        dev.e_main_off = d_sumoff.as<int>();
        dev.e_main_rows = d_sumcols.as<int>();
        dev.e_main_const = d_sumconst.as<double>();
        dev.e_corr_off = d_corroff.as<int>();
        dev.e_corr_rows = d_corrcols.as<int>();
        dev.e_corr_const = d_corrconst.as<double>();
        dev.pairs = d_pairs.as<CLPair>();
    }

    void build_device(bool have_noise, const std::vector<double> &chatM, const std::vector<double> &cfh,
                      const std::vector<BKMap> &bkm, const std::vector<double> &bnu, const std::vector<double> &bR,
                      const std::vector<double> &bdnu) {
        const int L = lmax - lmin + 1;
        // required map pairs (InitMapCls :997-1019, MapPair_to_Theory_i_j :284-299)
        pairs.clear();
        auto pair_index = [&](int i, int j) { return (i - 1) * i / 2 + (j - 1); };   // i >= j, 1-based
        for (int i = 1; i <= nreq; i++)
            for (int j = 1; j <= i; j++) {
                int f1 = map_fields[required_order[i - 1] - 1], f2 = map_fields[required_order[j - 1] - 1];
                if (f2 > f1) std::swap(f1, f2);
                CLPair p{};
                p.field = f1 * (f1 - 1) / 2 + (f2 - 1);
                p.cmb = (f1 <= 3 && f2 <= 3);
                p.fg = bk ? ((f1 == 2 && f2 == 2) ? 1 : (f1 == 3 && f2 == 3) ? 2 : 0)
                          : (smica && f1 == 1 && f2 == 1) ? 3 : 0;   // SMICA: CL%theory_i == 1 .and. CL%theory_j == 1
                p.mi = i - 1;
                p.mj = j - 1;
                pairs.push_back(p);
            }
        // window columns: one per (bin, window entry with an output); main then correction
        auto &cols = wcols;
        cols.clear();
        const int nE = nb * ncl;
        w_emain.assign(nE, {});
        w_ecorr.assign(nE, {});
        auto &e_main = w_emain, &e_corr = w_ecorr;
        auto add_windows = [&](const Windows &wn, std::vector<std::vector<int>> &lists) {
            const int norder = (int)wn.in_i.size();
            for (int b = 0; b < nb; b++)
                for (int k = 0; k < norder; k++) {
                    if (wn.out[k] <= 0) continue;
                    const double *Wk = &wn.W[((size_t)b * norder + k) * L];
                    HCol c{-1, L, -1, Wk, 0.0, false};
                    for (int l = 0; l < L; l++)
                        if (Wk[l] != 0.0) { c.lo = std::min(c.lo, l); c.hi = l; }
                    if (!wn.fix[k].empty()) {              // fix_cl: walker-independent dot
                        c.fixed = true;
                        for (int l = 0; l < L; l++) c.cst += Wk[l] * wn.fix[k][l];
                    } else {
                        if (wn.in_i[k] == 0 || wn.in_j[k] == 0)
                            fail(CMBL_ERR_FORMAT, "CMBlikes: bin window uses a spectrum of a map that is not required");
                        c.pair = pair_index(wn.in_i[k], wn.in_j[k]);
                    }
                    lists[(size_t)b * ncl + (wn.out[k] - 1)].push_back((int)cols.size());
                    cols.push_back(c);
                }
        };
        add_windows(bw, e_main);
        if (cw.present) add_windows(cw, e_corr);
        build_items();
        std::vector<int> e_to_x(nE, -1);
        for (int b = 0; b < nb; b++)
            for (int u = 0; u < ncl_used; u++) e_to_x[b * ncl + cl_use[u]] = b * ncl_used + u;
        std::vector<double> fc(nE, 0.0), noise(nE, 0.0);
        if (cw.present) fc = fidcorr;
        if (have_noise) noise = clnoise;

        auto up = [](DevBuf &d, const void *p, size_t bytes) {
            d.alloc(std::max<size_t>(bytes, 16));
            if (bytes) d.upload(p, bytes);
        };
        up(d_pairs, pairs.data(), pairs.size() * sizeof(CLPair));
        up(d_etox, e_to_x.data(), e_to_x.size() * 4);
        up(d_fidcorr, fc.data(), fc.size() * 8);
        up(d_noise, noise.data(), noise.size() * 8);
        up(d_chat, clhat.data(), clhat.size() * 8);
        up(d_cluse, cl_use.data(), cl_use.size() * 4);
        up(d_hlchat, chatM.data(), chatM.size() * 8);
        up(d_hlcf, cfh.data(), cfh.size() * 8);
        if (approx == 1) {   // the HL eigensolves' starting bases (cmbl_hl_rows_kernel warm start)
            const int n = nmaps;
            std::vector<double> u0((size_t)nb * n * n), v0((size_t)nb * n * n);
            for (int b = 0; b < nb; b++) {
                std::vector<double> cf(cfh.begin() + (size_t)b * n * n, cfh.begin() + (size_t)(b + 1) * n * n);
                std::vector<double> ev, U, cm = cf, R((size_t)n * n, 0.0), V;
                sym_eigen(cf, n, ev, U);                       // C_fid^1/2 and C_fid share eigenvectors
                bool ok = true;
                for (double e : ev) ok = ok && e > 0.0;
                if (ok) {
                    sym_power(cm, n, -1.0);                    // C_fid^-1/2
                    const double *ch = &chatM[(size_t)b * n * n];
                    std::vector<double> T((size_t)n * n, 0.0);
                    for (int i = 0; i < n; i++)
                        for (int j = 0; j < n; j++)
                            for (int k = 0; k < n; k++) T[i * n + j] += ch[i * n + k] * cm[k * n + j];
                    for (int i = 0; i < n; i++)
                        for (int j = 0; j < n; j++)
                            for (int k = 0; k < n; k++) R[i * n + j] += cm[i * n + k] * T[k * n + j];
                    sym_eigen(R, n, ev, V);
                } else {
                    U.assign((size_t)n * n, 0.0);
                    for (int i = 0; i < n; i++) U[i * n + i] = 1.0;
                    V = U;
                }
                std::copy(U.begin(), U.end(), u0.begin() + (size_t)b * n * n);
                std::copy(V.begin(), V.end(), v0.begin() + (size_t)b * n * n);
            }
            up(d_hlu0, u0.data(), u0.size() * 8);
            up(d_hlv0, v0.data(), v0.size() * 8);
        }
        if (bk) {
            up(d_bkmaps, bkm.data(), bkm.size() * sizeof(BKMap));
            up(d_bpnu, bnu.data(), bnu.size() * 8);
            up(d_bpR, bR.data(), bR.size() * 8);
            up(d_bpdnu, bdnu.data(), bdnu.size() * 8);
            std::vector<double> blnu(bnu.size()), ll80((lmax + 2) & ~1, 0.0);
            for (size_t k = 0; k < bnu.size(); k++) blnu[k] = std::log(bnu[k]);
            for (int l = 1; l < (int)ll80.size(); l++) ll80[l] = std::log(l / 80.0);
            up(d_bplnu, blnu.data(), blnu.size() * 8);
            up(d_logl80, ll80.data(), ll80.size() * 8);
            nsamp = (int)bnu.size();
        }
        qf.init(invcov, nX);
        up(d_invcov, invcov.data(), invcov.size() * 8);
        dev.lmin = lmin;
        dev.lmax = lmax;
        dev.pairs = d_pairs.as<CLPair>();
        dev.aberration = aberration;
        dev.cal_index = cal_index;
        dev.log_cal_prior = log_cal_prior;
        dev.nE = nE;
        dev.ncl_used = ncl_used;
        dev.nX = nX;
        dev.Np = qf.Np;
        dev.approx = approx;
        dev.has_corr = cw.present ? 1 : 0;
        dev.fidcorr = d_fidcorr.as<double>();
        dev.noise = d_noise.as<double>();
        dev.chat = d_chat.as<double>();
        dev.e_to_x = d_etox.as<int>();
        dev.bk = bk ? 1 : 0;
        dev.nreq = nreq;
        dev.LP = (lmax + 2) & ~1;
        dev.smica_pivot = 2000.0;
        dev.bkmaps = bk ? d_bkmaps.as<BKMap>() : nullptr;
        dev.bp_nu = bk ? d_bpnu.as<double>() : nullptr;
        dev.bp_lnu = bk ? d_bplnu.as<double>() : nullptr;
        dev.nsamp = bk ? nsamp : 0;
        dev.td_den = nullptr;   // per call, in the workspace (layout().td)
        dev.td0 = nullptr;
        dev.log_l80 = bk ? d_logl80.as<double>() : nullptr;
        dev.bp_R = bk ? d_bpR.as<double>() : nullptr;
        dev.bp_dnu = bk ? d_bpdnu.as<double>() : nullptr;
        hl.n = nmaps;
        hl.m = std::max(2, (nmaps + 1) & ~1);
        hl.nb = nb;
        hl.ncl = ncl;
        hl.ncl_used = ncl_used;
        hl.nX = nX;
        hl.Np = qf.Np;
        hl.chat = d_hlchat.as<double>();
        hl.cfhalf = d_hlcf.as<double>();
        hl.u0 = approx == 1 ? d_hlu0.as<double>() : nullptr;   // the warm-started eigensolves' bases
        hl.v0 = approx == 1 ? d_hlv0.as<double>() : nullptr;
        hl.cl_use = d_cluse.as<int>();
        hl.status = status_word();
    }

    // workspace: quadratic form | partial dots [rows][W] | C matrices [W][nE] (HL) |
    //            BK coef [W][3 nreq] + profiles [3][L][W] | addend [W]
    struct WsLayout { size_t part, cmat, coef, prof, add, td, total; };
    WsLayout layout(int W) const {
        auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
        WsLayout o{};
        o.part = al(qf.workspace_size(W));
        o.cmat = o.part + al((size_t)n_part_rows * W * 8);
        o.coef = o.cmat + al(approx == 1 ? (size_t)W * nb * ncl * 8 : 0);
        o.prof = o.coef + al(bk ? (size_t)W * 3 * nreq * 8 : 0);
        o.add = o.prof + al((bk || smica) ? (size_t)3 * dev.LP * W * 8 : 0);   // prof [W][3][LP]
        o.td = o.add + al((size_t)W * 8);
        o.total = o.td + al(bk ? (size_t)(nsamp + 1) * 8 : 0);   // T_dust table: td0, then nsamp denominators
        return o;
    }
    size_t workspace_size(int W) const override { return approx == 3 ? 256 : layout(W).total; }

    void loglike_batch(int W, const double *dl, long long ld_field, long long ld_walker, const double *nuis,
                       long long ld_nuis, double *out, void *ws, hipStream_t stream) override {
        run(W, dl, ld_field, ld_walker, nuis, ld_nuis, out, ws, stream, nullptr);
    }
    bool sparse_capable() const override { return approx != 3; }
    void loglike_batch_sparse(int W, const double *dl, long long ld_field, long long ld_walker, const double *nuis,
                              long long ld_nuis, double *out, void *ws, hipStream_t stream,
                              const int *wcount) override {
        run(W, dl, ld_field, ld_walker, nuis, ld_nuis, out, ws, stream, wcount);
    }

    // window stage: the direct path's work items (no BK foregrounds, no
    // aberration), one column per (item, window column) writing its partial row
    bool window_stage(WinStage &st) const override {
        if (approx == 3 || bk || smica || aberration != 0.0 || use_group || !binned) return false;
        st.kind = 0;
        st.cal_index = cal_index;
        st.cols.clear();
        for (size_t k = 0; k < h_items.size(); k++) {
            const WItem &it = h_items[k];
            const CLPair &pr = pairs[it.pair];
            for (size_t g = 0; g < h_item_cols[k].size(); g++) {
                const HCol &c = wcols[h_item_cols[k][g]];
                st.cols.push_back(WinCol{pr.field, it.l0, it.l1, c.W + (it.l0 - lmin), it.part + (int)g,
                                         (pr.cmb && cal_index >= 0) ? 1 : 0});
            }
        }
        return true;
    }
    double *window_out(void *ws, int W) const override {
        return reinterpret_cast<double *>(static_cast<char *>(ws) + layout(W).part);
    }
    QFDeferred after_window(int W, const double *nuis, long long ld_nuis, double *out, void *ws, hipStream_t stream,
                            bool defer, const SmallGaussLaunch *co = nullptr) override {
        if (co) fail(CMBL_ERR_ARG, "internal: %s carries no co-run", name.c_str());
        if (W <= 0) return QFDeferred{};
        if (n_nuis > 0 && !nuis) fail(CMBL_ERR_ARG, "%s needs its %d nuisance parameters", name.c_str(), n_nuis);
        if (defer && !deferred_capable()) fail(CMBL_ERR_UNSUPPORTED, "%s: no deferred evaluation", name.c_str());
        dev.wcount = nullptr;
        hl.wcount = nullptr;
        const double *nu = nuis ? nuis : reinterpret_cast<const double *>(ws);   // never read when n_nuis == 0
        return post_window(W, nu, ld_nuis, out, ws, stream, nullptr, defer);
    }
    // the small chi^2 as a co-run of another likelihood's deferred quadratic
    // form (the after_window stage of a fused small gaussian dataset)
    bool corun_small(SmallGaussLaunch &a, int W, const double *nuis, long long ld_nuis, double *out,
                     void *ws) override {
        if (!small_gauss || W <= 0 || !ws) return false;
        if (n_nuis > 0 && !nuis) fail(CMBL_ERR_ARG, "%s needs its %d nuisance parameters", name.c_str(), n_nuis);
        dev.wcount = nullptr;
        hl.wcount = nullptr;
        a = small_args(W, nuis ? nuis : reinterpret_cast<const double *>(ws), ld_nuis, out, ws);
        return true;
    }
    bool window_resegment(const std::map<int, std::vector<int>> &starts) override {
        if (approx == 3 || bk || smica || aberration != 0.0 || use_group || !binned) return false;
        const int L = lmax - lmin + 1;
        seg_starts.clear();
        for (auto &kv : starts) {
            std::vector<int> v{0};
            for (int c : kv.second)
                if (c - lmin > v.back() && c - lmin < L) v.push_back(c - lmin);
            seg_starts[kv.first] = v;
        }
        build_items();
        return true;
    }
    std::map<int, std::vector<int>> window_segments() const override { return seg_starts; }
    void window_set_segments(const std::map<int, std::vector<int>> &segs) override {
        if (seg_starts == segs) return;
        seg_starts = segs;
        build_items();
    }

    // the quadratic-form datasets (HL and large gaussian) can leave the combine to the sampler
    bool deferred_capable() const override { return approx != 3 && !small_gauss; }
    QFDeferred loglike_batch_deferred(int W, const double *dl, long long ld_field, long long ld_walker,
                                      const double *nuis, long long ld_nuis, void *ws, hipStream_t stream) override {
        if (!deferred_capable()) fail(CMBL_ERR_UNSUPPORTED, "%s: no deferred evaluation", name.c_str());
        if (!ws) fail(CMBL_ERR_ARG, "deferred evaluation needs a caller workspace");
        return run(W, dl, ld_field, ld_walker, nuis, ld_nuis, nullptr, ws, stream, nullptr, true);
    }

    QFDeferred run(int W, const double *dl, long long ld_field, long long ld_walker, const double *nuis,
                   long long ld_nuis, double *out, void *ws, hipStream_t stream, const int *wcount,
                   bool defer = false) {
        if (W <= 0) return QFDeferred{};
        dev.wcount = wcount;
        hl.wcount = wcount;
        if (n_nuis > 0 && !nuis) fail(CMBL_ERR_ARG, "%s needs its %d nuisance parameters", name.c_str(), n_nuis);
        if (ld_field < lmax + 1) fail(CMBL_ERR_ARG, "ld_field %lld < cl_lmax+1 = %d", ld_field, lmax + 1);
        if (W > 1 && ld_walker != 0 && ld_walker < (long long)(max_field + 1) * ld_field)
            fail(CMBL_ERR_ARG, "ld_walker must cover theory fields 0..%d", max_field);
        if (!ws) {
            own_ws.grow(workspace_size(W));
            ws = own_ws.p;
        }
        if (approx == 3) {
            timed_launch("cmbl_exact_kernel", stream, [&](hipEvent_t e0, hipEvent_t e1) {
                const dim3 g((W + EXACT_WPB - 1) / EXACT_WPB), bl(256);
                const double *nu = nuis ? nuis : dl;   // never read without a calibration parameter
                switch (nmaps) {
#define CMBL_EXACT(N)                                                                                     \
    case N:                                                                                               \
        hipExtLaunchKernelGGL(cmbl_exact_kernel<N>, g, bl, 0, stream, e0, e1, 0, xdev, dl, ld_field, ld_walker, \
                              nu, ld_nuis, out, W);                                                       \
        break;
                    CMBL_EXACT(1) CMBL_EXACT(2) CMBL_EXACT(3) CMBL_EXACT(4)
#undef CMBL_EXACT
                    default: break;
                }
            });
            HIP_CHECK(hipGetLastError());
            return QFDeferred{};
        }
        const WsLayout o = layout(W);
        char *base = static_cast<char *>(ws);
        double *partial = reinterpret_cast<double *>(base + o.part);
        double *coef = reinterpret_cast<double *>(base + o.coef);
        double *prof = reinterpret_cast<double *>(base + o.prof);
        const double *nu = nuis ? nuis : dl;   // never read when n_nuis == 0
        const int tiles = (W + 63) / 64;
        if (bk) {
            // the T_dust table is per call (this workspace), so concurrent calls on
            // other streams -- the sampler's walker groups -- cannot overwrite it
            dev.td0 = reinterpret_cast<double *>(base + o.td);
            dev.td_den = dev.td0 + 1;
            hipLaunchKernelGGL(cmbl_bk_tdtab, dim3((dev.nsamp + 255) / 256), dim3(256), 0, stream, dev, nu);
            HIP_CHECK(hipGetLastError());
            timed_launch("cmbl_bk_prologue", stream, [&](hipEvent_t e0, hipEvent_t e1) {
                hipExtLaunchKernelGGL(cmbl_bk_prologue, dim3(W), dim3(BKP_THREADS), 0, stream, e0, e1, 0, dev, nu, ld_nuis,
                                      coef, prof, W);
            });
            HIP_CHECK(hipGetLastError());
        }
        if (smica) {
            timed_launch("cmbl_smica_prologue", stream, [&](hipEvent_t e0, hipEvent_t e1) {
                hipExtLaunchKernelGGL(cmbl_smica_prologue, dim3((dev.LP + 255) / 256, W), dim3(256), 0, stream, e0, e1,
                                      0, dev, nu, ld_nuis, prof, W);
            });
            HIP_CHECK(hipGetLastError());
        }
        // 16-byte theory loads need aligned rows and even chunk starts
        bool vec_ok = ((reinterpret_cast<uintptr_t>(dl) & 15) == 0) && ld_field % 2 == 0 && ld_walker % 2 == 0 &&
                      items_even && (lmax + 1 < ld_field || (lmax % 2 == 1 && lmax + 1 <= ld_field));
        if (use_group) {
            const bool gvec = ((reinterpret_cast<uintptr_t>(dl) & 15) == 0) && ld_field % 2 == 0 && ld_walker % 2 == 0;
            static const int map_env = [] {   // A/B: CMAMD_WG_MAP=0 forces the item-per-XCD placement
                const char *e = std::getenv("CMAMD_WG_MAP");
                return e ? std::atoi(e) : 1;
            }();
            const int txcd = (map_env && tiles % 8 == 0) ? 1 : 0;
            const int nblk = txcd ? tiles * n_gitem : 8 * tiles * ((n_gitem + 7) / 8);
            timed_launch("cmbl_window_kernel", stream, [&](hipEvent_t e0, hipEvent_t e1) {
                if (dev.lform_dust != 0 || dev.lform_sync != 0)
                    hipExtLaunchKernelGGL(cmbl_window_group<true>, dim3(nblk), dim3(256), 0, stream, e0, e1, 0, dev,
                                          d_gitems.as<GItem>(), n_gitem, d_gw.as<double>(), dl, ld_field, ld_walker,
                                          nu, ld_nuis, (const double *)coef, (const double *)prof, dev.LP, partial, W,
                                          tiles, (int)gvec, txcd);
                else
                    hipExtLaunchKernelGGL(cmbl_window_group<false>, dim3(nblk), dim3(256), 0, stream, e0, e1, 0, dev,
                                          d_gitems.as<GItem>(), n_gitem, d_gw.as<double>(), dl, ld_field, ld_walker,
                                          nu, ld_nuis, (const double *)coef, (const double *)prof, dev.LP, partial, W,
                                          tiles, (int)gvec, txcd);
            });
        } else if (!bk && !smica && aberration == 0.0) {
            const int nblk = 8 * tiles * ((dev.nitem + 7) / 8);
            timed_launch("cmbl_window_kernel", stream, [&](hipEvent_t e0, hipEvent_t e1) {
                hipExtLaunchKernelGGL(cmbl_window_direct, dim3(nblk), dim3(256), 0, stream, e0, e1, 0, dev, dl,
                                      ld_field, ld_walker, nu, ld_nuis, partial, W, tiles, (int)vec_ok);
            });
        } else
        timed_launch("cmbl_window_kernel", stream, [&](hipEvent_t e0, hipEvent_t e1) {
#define CMBL_WINDOW(A, F)                                                                                        \
    hipExtLaunchKernelGGL(cmbl_window_kernel<A, F>, dim3(tiles, dev.nitem), dim3(256), 0, stream, e0, e1, 0, dev, dl, \
                          ld_field, ld_walker, nu, ld_nuis, (const double *)coef, (const double *)prof, partial, W,    \
                          (int)vec_ok)
            const bool ab = aberration != 0.0;
            if (bk || smica) {
                if (ab) CMBL_WINDOW(true, true);
                else CMBL_WINDOW(false, true);
            } else {
                if (ab) CMBL_WINDOW(true, false);
                else CMBL_WINDOW(false, false);
            }
#undef CMBL_WINDOW
        });
        HIP_CHECK(hipGetLastError());
        return post_window(W, nu, ld_nuis, out, ws, stream, wcount, defer);
    }

    void derived_batch(int W, const double *nuis, long long ld_nuis, double *out, long long ld_out,
                       hipStream_t stream) override {
        if (W <= 0 || n_derived <= 0) return;
        if (!out || ld_out < n_derived) fail(CMBL_ERR_ARG, "derived output needs %d columns", n_derived);
        if (!smica) return Like::derived_batch(W, nuis, ld_nuis, out, ld_out, stream);
        if (!nuis) fail(CMBL_ERR_ARG, "%s needs its %d nuisance parameters", name.c_str(), n_nuis);
        hipLaunchKernelGGL(cmbl_smica_derived, dim3((W + 63) / 64), dim3(64), 0, stream, dev,
                           pairs.empty() ? 0 : (int)(pairs[0].fg == 3), nuis, ld_nuis, out, ld_out, n_derived, W);
        HIP_CHECK(hipGetLastError());
    }

    SmallGaussLaunch small_args(int W, const double *nu, long long ld_nuis, double *out, void *ws) const {
        SmallGaussLaunch a{};
        a.d = SmallGaussDev{dev.nE,        dev.nX,         dev.has_corr,       dev.cal_index, dev.log_cal_prior,
                            dev.e_to_x,    dev.e_main_const, dev.e_corr_const, dev.fidcorr,   dev.chat,
                            sdev.ntask,    sdev.trow,      sdev.e_main_t,      sdev.e_corr_t, dev.wcount};
        a.partial = reinterpret_cast<const double *>(static_cast<const char *>(ws) + layout(W).part);
        a.nuis = nu;
        a.ld_nuis = ld_nuis;
        a.M = d_invcov.as<double>();
        a.out = out;
        a.W = W;
        return a;
    }

    // the kernels after the window stage: binned spectra, then chi^2 (small
    // gaussian) or the HL transform / gaussian residuals and the quadratic form
    QFDeferred post_window(int W, const double *nu, long long ld_nuis, double *out, void *ws, hipStream_t stream,
                           const int *wcount, bool defer) {
        const WsLayout o = layout(W);
        char *base = static_cast<char *>(ws);
        void *qws = ws;
        double *partial = reinterpret_cast<double *>(base + o.part);
        double *cmat = reinterpret_cast<double *>(base + o.cmat);
        double *addend = reinterpret_cast<double *>(base + o.add);
        const bool use_add = log_cal_prior > 0 && cal_index >= 0;
        const int tiles = (W + 63) / 64;
        if (small_gauss) {
            const SmallGaussLaunch a = small_args(W, nu, ld_nuis, out, ws);
            timed_launch("cmbl_gauss_small_kernel", stream, [&](hipEvent_t e0, hipEvent_t e1) {
                const int ng = (W + SMALL_WT - 1) / SMALL_WT;
                hipExtLaunchKernelGGL(cmbl_gauss_small_kernel<SMALL_WT>, dim3(small_gauss_blocks(ng)), dim3(256), 0,
                                      stream, e0, e1, 0, a, ng);
            });
            HIP_CHECK(hipGetLastError());
            return QFDeferred{};
        }
        timed_launch("cmbl_reduce_kernel", stream, [&](hipEvent_t e0, hipEvent_t e1) {
            hipExtLaunchKernelGGL(cmbl_reduce_kernel, dim3(tiles, (dev.nE + 3) / 4), dim3(256), 0, stream, e0, e1, 0, dev,
                                  (const double *)partial, nu, ld_nuis, qf.x_rows(qws), cmat, use_add ? addend : nullptr,
                                  qf.counters(qws, W), qf.n_counters(W), W);
        });
        HIP_CHECK(hipGetLastError());
        if (approx == 1) {
            timed_launch("cmbl_hl_kernel", stream, [&](hipEvent_t e0, hipEvent_t e1) {
                const dim3 bl(64);
                switch (hl.m) {
#define CMBL_HLR(MM)                                                                                              \
    case MM:                                                                                                      \
        hipExtLaunchKernelGGL(cmbl_hl_rows_kernel<MM>, dim3((W * nb + 64 / MM - 1) / (64 / MM)), bl, 0, stream,    \
                              e0, e1, 0, hl, (const double *)cmat, qf.x_rows(qws), W);                           \
        break;
                    CMBL_HLR(2) CMBL_HLR(4) CMBL_HLR(6) CMBL_HLR(8) CMBL_HLR(10) CMBL_HLR(12) CMBL_HLR(14)
                    CMBL_HLR(16)
#undef CMBL_HLR
                    default: break;
                }
            });
            HIP_CHECK(hipGetLastError());
        }
        if (defer) return qf.launch_deferred(W, qws, use_add ? addend : nullptr, stream, "cmbl_quadform");
        qf.launch(W, qws, use_add ? addend : nullptr, out, stream, "cmbl_quadform", wcount);
        return QFDeferred{};
    }
};

std::unique_ptr<Like> make_cmblikes(const Ini &ini, const std::string &tag) {
    return std::unique_ptr<Like>(new CMBLikes(ini, tag));
}

}  // namespace cmamd

#ifdef CMAMD_STAMPS
extern "C" int cmamd_debug_hl_sweeps(unsigned int *host) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(cmamd::g_hl_sweeps), sizeof(cmamd::g_hl_sweeps)) == hipSuccess ? 0 : -5;
}
extern "C" int cmamd_debug_hl_phase(unsigned long long *host) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(cmamd::g_hl_phase), sizeof(cmamd::g_hl_phase)) == hipSuccess ? 0 : -5;
}
extern "C" int cmamd_debug_hl_tp(unsigned long long *host) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(cmamd::g_hl_tp), sizeof(cmamd::g_hl_tp)) == hipSuccess ? 0 : -5;
}
#endif
