// SPTpol bandpower likelihoods (reference TSPTpolEELike, source/CMB_SPTpol_TEEE_2017.f90,
// and TSPTpolBBLike, source/CMB_SPTpol_BB_2019.f90) batched over W walkers on
// MI355X (gfx950).
//
// Per walker, for every band k (TE, EE  |  150x150, 95x150, 95x95):
//   dl_fgs_k(l) = theory + foregrounds         (TEEE :397-449, BB :497-533)
//   tmpcb_k     = W_k^T dl_fgs_k / Cal_k        (dgemv 'T', TEEE :477-484, BB :557-563)
//   delta       = tmpcb * BeamFac - spec        (TEEE :500-513, BB :576-598)
//   -lnL        = sum log L_ii + delta^T C^-1 delta / 2 + priors
//                 (Matrix_GaussianLogLikeCholDouble, TEEE :628-665; priors :525-564 / :620-652)
//
// Kernels (same stream):
//   sptpol_window_kernel<KIND, ABER>  the W_k^T dl_fgs_k contraction as a skinny
//       GEMM on the f64 MFMA.  A work item is (band, <= 16 window columns, <= SP_CH
//       l); the l range of an item is the union of its columns' non-zero window
//       support, so the dense on-disk windows cost only their support.  A
//       256-thread workgroup takes 64 walkers x one item: the item's weights and
//       per-l tables go HBM/L2 -> LDS once, each lane forms dl_fgs for 8
//       consecutive l of its walker in registers (foregrounds, derivative and
//       aberration from the l-1 / l+8 halo) and feeds v_mfma_f64_16x16x4f64.
//       Theory for the next 32 l is in flight across the current MFMAs.
//   sptpol_delta_kernel  sums each bandpower's item partials in fixed order
//       (one wave per bandpower, 64 walkers per wave), applies 1/Cal, the beam
//       factors and the data, writes delta rows for the quadratic form (LDS
//       transpose) and the log-det + prior addend; zeroes the tickets.
//   quadform_ksplit      delta^T C^-1 delta / 2 + addend (quadform.hip).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <sstream>

#include "quadform.h"

namespace cmamd {

static constexpr int SP_COLS = 16;      // window columns per item (one MFMA block)
static constexpr int SP_STEP = 32;      // l per MFMA step (4 lane groups x 8 l)
static constexpr int SP_CH = 256;       // l per item (8 steps)
static constexpr int SP_DB = 8;         // bandpowers per delta-kernel block (one wave each)
static constexpr double SP_TWOPI = 6.283185307179586476925286766559;

typedef double f64x4 __attribute__((ext_vector_type(4)));

enum { SP_TEEE = 0, SP_BB = 1 };

struct SPItem {
    int k;          // band
    int l0;         // first l (even)
    int nstep;      // steps of SP_STEP l
    int ncol;       // columns (<= 16)
    int part;       // first partial row
    int pad;
    long long woff; // weights [16][nstep * SP_STEP] (zero padded)
    long long toff; // per-l tables [nstep * SP_STEP + 2][4], from l = l0 - 1
};

struct SPDev {
    int nitem, lmin, lmax;
    const SPItem *items;
    const double *wts;
    const double *tabs;
    int field[3];            // theory field of each band
    double dust_scale[3];    // BB: dustFreqScalingFrom150GHz(effFreqs(:,k))
    double blind_abb;        // BB
    // delta / prior stage
    int nall, nbin, nband, Np, nbeam;
    const int *row_off, *rows;      // partial rows per bandpower
    const double *beam_err;         // [nbeam][nall]
    const double *spec;             // [nall] data in delta order
    double logdet;
    // priors (TEEE: Tcal, Pcal, kappa, alphaTE, alphaEE; BB: cal (2x2), Add)
    int pr_on[5];
    double pr_mean[5], pr_sigma[5];
    double inv_cal[3];              // BB InvCalCov(1,1), (1,2), (2,2)
};

// Per-l tables (host-computed with the reference's expressions):
//   TEEE: [rawspec_factor, cl_to_dl_conversion, deriv_factor, log(l/80)]   (:202-211)
//   BB:   [Dls_poisson, Dls_galdust, Dls_tensor, 0]                          (:226-228, :419-433)
template <int KIND, bool ABER>
__global__ __launch_bounds__(256) void sptpol_window_kernel(SPDev c, const double *__restrict__ dl, long long ld_field,
                                                            long long ld_walker, const double *__restrict__ nuis,
                                                            long long ld_nuis, double *__restrict__ partial, int W,
                                                            int tiles, int vec_ok)
{
    constexpr int LPL = 8;
    constexpr int WROW = SP_CH + 2;            // LDS row stride of the weights (doubles)
    __shared__ __attribute__((aligned(16))) double wsh[SP_COLS * WROW];
    __shared__ __attribute__((aligned(16))) double tsh[(SP_CH + 2) * 4];
    // blocks are dealt to the XCDs round-robin: all walker tiles of an item on one XCD
    // (its weights in one L2); measured faster than an XCD-balanced split of the units
    const int b = blockIdx.x, xcd = b & 7, j = b >> 3;
    const int item = xcd + 8 * (j / tiles), tile = j % tiles;
    if (item >= c.nitem) return;
    const SPItem it = c.items[item];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int li = lane & 15, kq = lane >> 4;
    const int w = tile * 64 + wave * 16 + li;
    const int wl = min(w, W - 1);
    const int L = it.nstep * SP_STEP;
    // weights and tables -> LDS (all loads in flight, one barrier)
    {
        const double2 *src = reinterpret_cast<const double2 *>(c.wts + it.woff);
        const int n2 = SP_COLS * L / 2;
        for (int q = tid; q < n2; q += 256) {
            const int col = (2 * q) / L, l = (2 * q) % L;
            *reinterpret_cast<double2 *>(wsh + col * WROW + l) = src[q];
        }
        const double2 *ts = reinterpret_cast<const double2 *>(c.tabs + it.toff);
        for (int q = tid; q < (L + 2) * 2; q += 256) reinterpret_cast<double2 *>(tsh)[q] = ts[q];
    }
    const double *Df = dl + (long long)wl * ld_walker + (long long)c.field[it.k] * ld_field;
    const double *P = nuis + (long long)wl * ld_nuis;
    // per-walker foreground parameters of this band
    double p0, p1, p2, p3;
    if (KIND == SP_TEEE) {
        // iKappa=1, iPS_TE=2, iPS_EE=3, iDust_TE=4, iDustAlpha_TE=5, iDust_EE=6, iDustAlpha_EE=7 (:398)
        p0 = P[0];                                             // kappa
        p1 = P[1 + it.k] / (3000 * 3001 / SP_TWOPI);           // PoissonLevels(k) (:426)
        p2 = P[3 + 2 * it.k];                                  // ADust(k)
        p3 = P[4 + 2 * it.k] + 2.0;                            // alphaDust(k) + 2
    } else {
        // iAbb=1, iR=2, iConstbb=3, iAdd=4, iPoisson150..90 = 5..7 (:470-474)
        const double abb = P[0];
        p0 = abb != 1.0 ? abb + c.blind_abb : 1.0;             // dls *= (Abb + blind) if Abb /= 1 (:484-486)
        if (abb == 0.0) p0 = 0.0;                              // dls = 0 if Abb == 0 (:487-488)
        p1 = P[2];                                             // constant
        p2 = P[1];                                             // r
        p3 = P[4 + it.k];                                      // PoissonLevels(k)
    }
    const double addust = KIND == SP_BB ? P[3] : 0.0;
    const double dsc = KIND == SP_BB ? c.dust_scale[it.k] : 0.0;
    // theory of one step: this lane's 8 l (and the l-1 / l+8 halo for TEEE)
    double t[LPL + 2], tn[LPL + 2];
    // l beyond lmax + 1 (padding of the last step) reads as 0: the caller's rows
    // need only hold l <= lmax + 1 (ClArray into dls(1:lmax+1), :388)
    const int lcap = c.lmax + 1;
    auto load_t = [&](int st, double *dst) {
        const int lb = it.l0 + st * SP_STEP + LPL * kq;
        if (vec_ok && lb + LPL - 1 <= lcap) {
            const double2 *src = reinterpret_cast<const double2 *>(Df + lb);
#pragma unroll
            for (int s = 0; s < LPL / 2; s++) {
                const double2 v = src[s];
                dst[1 + 2 * s] = v.x;
                dst[2 + 2 * s] = v.y;
            }
        } else {
#pragma unroll
            for (int s = 0; s < LPL; s++) dst[1 + s] = lb + s <= lcap ? Df[lb + s] : 0.0;
        }
        if (KIND == SP_TEEE) {
            dst[0] = Df[lb - 1];
            dst[LPL + 1] = lb + LPL <= lcap ? Df[lb + LPL] : 0.0;
        }
    };
    f64x4 acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
    load_t(0, t);
    __syncthreads();
    for (int st = 0; st < it.nstep; st++) {
        const bool more = st + 1 < it.nstep;
        if (more) load_t(st + 1, tn);                      // in flight across this step's MFMAs
        const int lr = st * SP_STEP + LPL * kq;            // l - l0 of the lane's first l
        double v[LPL];
        if (KIND == SP_TEEE) {
            double raw[LPL + 2];
#pragma unroll
            for (int s = 0; s < LPL + 2; s++) raw[s] = tsh[4 * (lr + s)] * t[s];   // rawspec_factor * dls (:407)
#pragma unroll
            for (int s = 0; s < LPL; s++) {
                const double *tb = tsh + 4 * (lr + s + 1);
                const double l = (double)(it.l0 + lr + s);
                const double deriv = tb[2] * (raw[s + 2] - raw[s]);                    // :411
                double f = (p1 - p0 * deriv) * tb[1];                                  // :431
                f = f + t[s + 1];                                                      // :434
                if (ABER) {
                    double a = (t[s + 2] - t[s]) / 2.;                                 // :419
                    a = (-1 * (double)0.0012309f * (double)-0.4033f) * l * a;          // :420
                    f = f + a;                                                         // :436
                }
                f = f + p2 * exp(p3 * tb[3]);                                          // Adust (l/80)^(alpha+2) (:439)
                v[s] = (l >= c.lmin && l <= c.lmax) ? f : 0.0;
            }
        } else {
#pragma unroll
            for (int s = 0; s < LPL; s++) {
                const double *tb = tsh + 4 * (lr + s + 1);
                double x = t[s + 1] * p0;                                              // :484-488
                if (p0 == 0.0) x = 0.0;
                x = x + p1;                                                            // :492
                x = x + p2 * tb[2];                                                    // :498
                double f = p3 * tb[0];                                                 // :533
                f = f + (addust * tb[1]) * dsc;                                        // :537
                f = f + x;                                                             // :541
                const int l = it.l0 + lr + s;
                v[s] = (l >= c.lmin && l <= c.lmax) ? f : 0.0;
            }
        }
        double a[LPL];
        {
            const double *src = wsh + li * WROW + lr;
#pragma unroll
            for (int s = 0; s < LPL / 2; s++) {
                const double2 q = *reinterpret_cast<const double2 *>(src + 2 * s);
                a[2 * s] = q.x;
                a[2 * s + 1] = q.y;
            }
        }
#pragma unroll
        for (int s = 0; s < LPL; s += 2) {
            acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], v[s], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s + 1], v[s + 1], acc1, 0, 0, 0);
        }
        if (more) {
#pragma unroll
            for (int s = 0; s < LPL + 2; s++) t[s] = tn[s];
        }
    }
    if (w < W) {
        // D: walker = lane & 15, column = (lane >> 4) + 4 r
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int col = kq + 4 * r;
            if (col < it.ncol) partial[(long long)(it.part + col) * W + w] = acc0[r] + acc1[r];
        }
    }
}

// tmpcb / Cal, * BeamFac, - spec -> delta rows [W][Np]; addend = log det + priors.
// Block = 64 walkers x SP_DB bandpowers, one wave per bandpower: each lane sums
// its walker's partial rows (coalesced across the wave, eight loads in flight,
// added in row order), the block transposes through LDS and writes SP_DB
// consecutive delta entries per walker row.  Block (0, 0) zeroes the
// quadratic-form tickets; bandpower group 0 writes the addend.
template <int KIND>
__global__ __launch_bounds__(64 * SP_DB) void sptpol_delta_kernel(SPDev c, const double *__restrict__ partial,
                                                                  const double *__restrict__ nuis, long long ld_nuis,
                                                                  double *__restrict__ xrows, double *__restrict__ addend,
                                                                  unsigned int *__restrict__ counters, int n_counters,
                                                                  int W)
{
    __shared__ double tile[64][SP_DB + 1];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int w = blockIdx.x * 64 + lane;
    const int i = blockIdx.y * SP_DB + wave;
    if (blockIdx.x == 0 && blockIdx.y == 0)
        for (int q = tid; q < n_counters; q += 64 * SP_DB) counters[q] = 0u;
    double v = 0.0;
    if (i < c.nall && w < W) {
        const double *P = nuis + (long long)w * ld_nuis;
        const int r0 = c.row_off[i], r1 = c.row_off[i + 1];
        double s = 0.0;
        for (int r = r0; r < r1; r += 8) {
            double t[8];
#pragma unroll
            for (int u = 0; u < 8; u++) t[u] = r + u < r1 ? partial[(long long)c.rows[r + u] * W + w] : 0.0;
#pragma unroll
            for (int u = 0; u < 8; u++) s += t[u];
        }
        const int k = i / c.nbin;
        double cal;
        if (KIND == SP_TEEE) {
            const double tc = P[7], pc = P[8];                 // CalFactors(k+1) = Tcal^2 Pcal^k (:455-457)
            cal = (tc * tc) * (k == 0 ? pc : pc * pc);
        } else {
            const double b150 = P[7], b90 = P[8];              // :507-509
            cal = k == 0 ? b150 * b150 : (k == 1 ? b90 * b150 : b90 * b90);
        }
        s = s / cal;
        double bf = 1.0;                                       // BeamFac (:500-503)
        for (int t = 0; t < c.nbeam; t++) bf = bf * (1 + c.beam_err[t * c.nall + i] * P[9 + t]);
        v = s * bf - c.spec[i];
    }
    tile[lane][wave] = v;
    __syncthreads();
    {
        const int wl = tid / SP_DB, q = tid % SP_DB;
        const int ww = blockIdx.x * 64 + wl, ii = blockIdx.y * SP_DB + q;
        if (ww < W && ii < c.Np) xrows[(long long)ww * c.Np + ii] = tile[wl][q];
    }
    if (blockIdx.y == 0 && wave == 0 && w < W) {
        const double *P = nuis + (long long)w * ld_nuis;
        double pr = 0.0;
        for (int t = 0; t < c.nbeam; t++) pr += P[9 + t] * P[9 + t];
        pr = 0.5 * pr;
        if (KIND == SP_TEEE) {
            const int ix[5] = {7, 8, 0, 4, 6};                     // Tcal, Pcal, kappa, alphaTE, alphaEE
            for (int q = 0; q < 5; q++) {
                if (!c.pr_on[q]) continue;
                const double t = q < 2 ? log(P[ix[q]] / c.pr_mean[q]) / c.pr_sigma[q]
                                       : (P[ix[q]] - c.pr_mean[q]) / c.pr_sigma[q];
                pr = pr + 0.5 * (t * t);
            }
        } else {
            if (c.pr_on[0]) {
                const double y1 = log(P[8]), y2 = log(P[7]);
                pr = pr + 0.5 * (c.inv_cal[0] * y1 * y1 + 2 * c.inv_cal[1] * y1 * y2 + c.inv_cal[2] * y2 * y2);
            }
            if (c.pr_on[1]) {
                const double t = (P[3] - c.pr_mean[1]) / c.pr_sigma[1];
                pr = pr + 0.5 * (t * t);
            }
        }
        addend[w] = c.logdet + pr;
    }
}

// ------------------------------------------------------------------ host side

namespace {

std::vector<std::string> read_lines(const std::string &path) {
    std::ifstream f(path);
    if (!f) fail(CMBL_ERR_IO, "SPTpol: cannot read %s", path.c_str());
    std::vector<std::string> out;
    std::string s;
    while (std::getline(f, s)) out.push_back(s);
    return out;
}

double num(const std::string &tok) {
    std::string t = tok;
    for (auto &ch : t)
        if (ch == 'd' || ch == 'D') ch = 'e';
    try {
        return std::stod(t);
    } catch (...) {
        fail(CMBL_ERR_FORMAT, "SPTpol: bad number '%s'", tok.c_str());
    }
}

// list-directed read of the n-th field of a record
double field(const std::string &line, size_t n, const std::string &path) {
    std::string t = line;
    for (auto &ch : t)
        if (ch == ',') ch = ' ';
    auto toks = split_ws(t);
    if (toks.size() <= n) fail(CMBL_ERR_FORMAT, "SPTpol: short record in %s: '%s'", path.c_str(), line.c_str());
    return num(toks[n]);
}

bool logical(const Ini &ini, const std::string &key) {   // Ini%Read_Logical(key, .false.)
    std::string v = ini.str(key);
    if (v.empty()) return false;
    const char ch = (char)std::toupper(v[0] == '.' && v.size() > 1 ? v[1] : v[0]);
    if (ch == 'T' || ch == '1' || ch == 'Y') return true;
    if (ch == 'F' || ch == '0' || ch == 'N') return false;
    fail(CMBL_ERR_FORMAT, "SPTpol: bad logical %s = %s", key.c_str(), v.c_str());
}

double real4(const Ini &ini, const std::string &key, float def) {   // Ini%Read_Real: a REAL(4)
    std::string v = ini.str(key);
    if (v.empty()) return (double)def;
    for (auto &ch : v)
        if (ch == 'd' || ch == 'D') ch = 'e';
    return (double)std::strtof(v.c_str(), nullptr);
}

std::string required_path(const Ini &ini, const std::string &key) {   // Read_String_Default(key, '')
    std::string v = ini.str(key);
    if (v.empty()) fail(CMBL_ERR_FORMAT, "Missing required sptpol key: %s", key.c_str());
    return v;
}

std::vector<char> read_bytes(const std::string &path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) fail(CMBL_ERR_IO, "SPTpol: cannot read %s", path.c_str());
    return std::vector<char>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

// OpenReadBinaryFile(recl = n*8) + read(rec=i) cov(:,i): n x n doubles, record i = column i
std::vector<double> read_direct_matrix(const std::string &path, int n) {
    auto b = read_bytes(path);
    if (b.size() < (size_t)n * n * 8) fail(CMBL_ERR_FORMAT, "SPTpol: %s holds fewer than %d x %d doubles", path.c_str(), n, n);
    std::vector<double> colmajor((size_t)n * n), M((size_t)n * n);
    std::memcpy(colmajor.data(), b.data(), (size_t)n * n * 8);
    for (int i = 0; i < n; i++)            // column i -> row-major M[r][i]
        for (int r = 0; r < n; r++) M[(size_t)r * n + i] = colmajor[(size_t)i * n + r];
    return M;
}

// dpotrf 'L' (Matrix_CholeskyDouble) -> sum log L_ii, the log-det term of
// Matrix_GaussianLogLikeCholDouble
double chol_logdet(std::vector<double> A, int n) {
    double ld = 0.0;
    for (int j = 0; j < n; j++) {
        double d = A[(size_t)j * n + j];
        for (int k = 0; k < j; k++) d -= A[(size_t)j * n + k] * A[(size_t)j * n + k];
        if (!(d > 0.0)) fail(CMBL_ERR_NUMERIC, "Matrix_CholeskyDouble: not positive definite %d", j + 1);
        d = std::sqrt(d);
        A[(size_t)j * n + j] = d;
        for (int i = j + 1; i < n; i++) {
            double s = A[(size_t)i * n + j];
            for (int k = 0; k < j; k++) s -= A[(size_t)i * n + k] * A[(size_t)j * n + k];
            A[(size_t)i * n + j] = s / d;
        }
        ld += std::log(d);
    }
    return ld;
}

// dBdT / Bnu / dustFreqScalingFrom150GHz (CMB_SPTpol_BB_2019.f90:761-813); the
// REAL(4) literals of the reference are kept as floats promoted to double.
double dBdT(double nu, double nu0) {
    const double x0 = nu0 / (double)56.78f;
    const double dBdT0 = std::pow(x0, 4) * std::exp(x0) / std::pow(std::exp(x0) - 1, 2);
    const double x = nu / (double)56.78f;
    return std::pow(x, 4) * std::exp(x) / std::pow(std::exp(x) - 1, 2) / dBdT0;
}
double Bnu(double nu, double nu0, double T) {
    const double hk = (double)4.799237e-2f;
    double b = std::pow(nu / nu0, 3);
    return b * (std::exp(hk * nu0 / T) - 1.0) / (std::exp(hk * nu / T) - 1.0);
}
double dust_scaling(double f1, double f2) {
    const double beta = (double)1.59f, Tdust = (double)19.6f;
    double s = std::pow((f1 * f2) / (150.0 * 150.0), beta);
    s = s * Bnu(f1, 150.0, Tdust) * Bnu(f2, 150.0, Tdust);
    return s / dBdT(f1, 150.0) / dBdT(f2, 150.0);
}

}  // namespace

struct SPTpol final : Like {
    int kind = SP_TEEE;
    int lmin = 0, lmax = 0, nbin = 0, nband = 0, nall = 0, nbeam = 0, need_lmax = 0;
    bool aberration = false;
    QuadForm qf;
    SPDev dev{};
    int n_part_rows = 0;
    DevBuf d_items, d_wts, d_tabs, d_rowoff, d_rows, d_beam, d_spec;

    SPTpol(const Ini &ini, const std::string &tg) {
        tag = tg;
        kind = tg == "SPTPOL_BB" ? SP_BB : SP_TEEE;
        name = ini.str("name", kind == SP_BB ? "SPTpol_BB_2019" : "SPTpol_TEEE_2017");
        if (kind == SP_TEEE) read_teee(ini);
        else read_bb(ini);
    }

    // windows [lmax-lmin+1][nall] (row l), cov row-major nall^2, spec[nall],
    // beam [nbeam][nall], tables [NL + 4][4] from l = lmin - 2 (zero outside lmin-1 .. lmax+1)
    void finish(const std::vector<double> &win, std::vector<double> cov, const std::vector<double> &spec,
                const std::vector<double> &beam, const std::vector<double> &tab, int fields[3]) {
        const int NL = lmax - lmin + 1;
        dev.logdet = chol_logdet(cov, nall);
        spd_inverse(cov, nall);
        qf.init(cov, nall);
        // work items: per band, groups of <= 16 consecutive columns over the union of
        // their non-zero support, cut into <= SP_CH l
        std::vector<SPItem> items;
        std::vector<double> wts, tabs;
        std::vector<std::vector<int>> col_rows(nall);
        int part = 0;
        for (int k = 0; k < nband; k++) {
            for (int c0 = 0; c0 < nbin; c0 += SP_COLS) {
                const int nc = std::min(SP_COLS, nbin - c0);
                int a = NL, z = -1;
                for (int c = 0; c < nc; c++) {
                    const int col = k * nbin + c0 + c;
                    for (int l = 0; l < NL; l++)
                        if (win[(size_t)l * nall + col] != 0.0) {
                            a = std::min(a, l);
                            z = std::max(z, l);
                        }
                }
                if (z < a) continue;   // all-zero windows: the bandpowers are 0 (no partial rows)
                const int la = (lmin + a) & ~1;   // even first l: 16-byte theory loads (>= lmin - 1)
                const int lz = lmin + z;
                for (int s0 = la; s0 <= lz; s0 += SP_CH) {
                    const int len = std::min(SP_CH, lz - s0 + 1);
                    SPItem it{};
                    it.k = k;
                    it.l0 = s0;
                    it.nstep = (len + SP_STEP - 1) / SP_STEP;
                    it.ncol = nc;
                    it.part = part;
                    it.woff = (long long)wts.size();
                    it.toff = (long long)tabs.size();
                    const int Lp = it.nstep * SP_STEP;
                    for (int c = 0; c < SP_COLS; c++)
                        for (int l = 0; l < Lp; l++) {
                            const int ix = s0 + l - lmin;
                            wts.push_back(c < nc && ix >= 0 && ix < NL ? win[(size_t)ix * nall + k * nbin + c0 + c] : 0.0);
                        }
                    for (int l = 0; l < Lp + 2; l++) {          // l = l0 - 1 .. l0 + Lp
                        const int q = s0 - 1 + l - (lmin - 2);  // tab[q] <-> l = lmin - 2 + q
                        for (int u = 0; u < 4; u++) tabs.push_back(q < NL + 4 ? tab[(size_t)q * 4 + u] : 0.0);
                    }
                    for (int c = 0; c < nc; c++) col_rows[k * nbin + c0 + c].push_back(part + c);
                    part += nc;
                    items.push_back(it);
                }
            }
        }
        n_part_rows = part;
        std::vector<int> roff(nall + 1, 0), rows;
        for (int i = 0; i < nall; i++) {
            for (int r : col_rows[i]) rows.push_back(r);
            roff[i + 1] = (int)rows.size();
        }
        if (rows.empty()) rows.push_back(0);
        need_lmax = lmax + 1;     // dls(1:lmax+1) (ClArray into dimension(spt_windows_lmax+1))
        d_items.alloc(std::max<size_t>(1, items.size()) * sizeof(SPItem));
        if (!items.empty()) d_items.upload(items.data(), items.size() * sizeof(SPItem));
        d_wts.alloc(std::max<size_t>(1, wts.size()) * 8);
        if (!wts.empty()) d_wts.upload(wts.data(), wts.size() * 8);
        d_tabs.alloc(std::max<size_t>(1, tabs.size()) * 8);
        if (!tabs.empty()) d_tabs.upload(tabs.data(), tabs.size() * 8);
        d_rowoff.alloc(roff.size() * 4);
        d_rowoff.upload(roff.data(), roff.size() * 4);
        d_rows.alloc(rows.size() * 4);
        d_rows.upload(rows.data(), rows.size() * 4);
        d_beam.alloc(std::max<size_t>(1, beam.size()) * 8);
        if (!beam.empty()) d_beam.upload(beam.data(), beam.size() * 8);
        d_spec.alloc(spec.size() * 8);
        d_spec.upload(spec.data(), spec.size() * 8);
        dev.nitem = (int)items.size();
        dev.lmin = lmin;
        dev.lmax = lmax;
        dev.items = d_items.as<SPItem>();
        dev.wts = d_wts.as<double>();
        dev.tabs = d_tabs.as<double>();
        for (int k = 0; k < 3; k++) dev.field[k] = fields[k];
        dev.nall = nall;
        dev.nbin = nbin;
        dev.nband = nband;
        dev.Np = qf.Np;
        dev.nbeam = nbeam;
        dev.row_off = d_rowoff.as<int>();
        dev.rows = d_rows.as<int>();
        dev.beam_err = d_beam.as<double>();
        dev.spec = d_spec.as<double>();
    }

    void read_teee(const Ini &ini) {           // SPTpol_TEEE_ReadIni / InitSPTpolData (:56-352)
        const bool EEonly = logical(ini, "sptpol_EEonly"), TEonly = logical(ini, "sptpol_TEonly");
        aberration = logical(ini, "correct_aberration");
        dev.pr_on[0] = logical(ini, "sptpol_tcal_prior");
        dev.pr_mean[0] = real4(ini, "sptpol_meanTcal", 1.0f);
        dev.pr_sigma[0] = std::log(1 + real4(ini, "sptpol_sigmaTcal", 0.005f));
        dev.pr_on[1] = logical(ini, "sptpol_pcal_prior");
        dev.pr_mean[1] = real4(ini, "sptpol_meanPcal", 1.0f);
        (void)real4(ini, "sptpol_sigmaPcal", 0.02f);
        dev.pr_sigma[1] = std::log(1 + dev.pr_sigma[0]);      // :79 sigmaPcal = log(1+sigmaTcal) (sic)
        dev.pr_on[2] = logical(ini, "sptpol_kappa_prior");
        dev.pr_mean[2] = real4(ini, "sptpol_meankappa", 0.0f);
        dev.pr_sigma[2] = real4(ini, "sptpol_sigmakappa", 0.001f);
        dev.pr_on[4] = logical(ini, "sptpol_alphaEE_prior");
        dev.pr_mean[4] = real4(ini, "sptpol_meanAlphaEE", -2.42f);
        dev.pr_sigma[4] = real4(ini, "sptpol_sigmaAlphaEE", 0.02f);
        dev.pr_on[3] = logical(ini, "sptpol_alphaTE_prior");
        dev.pr_mean[3] = real4(ini, "sptpol_meanAlphaTE", -2.42f);
        dev.pr_sigma[3] = real4(ini, "sptpol_sigmaAlphaTE", 0.02f);
        nuisance_names = load_paramnames(required_path(ini, "sptpol_TEEE_params_file"), &n_nuis);
        if (n_nuis < 11)
            fail(CMBL_ERR_FORMAT, "SPTPOL_TEEE needs 11 nuisance parameters (kappa .. beam factors), got %d", n_nuis);
        if (logical(ini, "print_spectrum")) fail(CMBL_ERR_UNSUPPORTED, "SPTpol print_spectrum is not supported");
        const std::string desc = required_path(ini, "sptpol_TEEE_desc_file");
        const std::string bpf = required_path(ini, "sptpol_TEEE_bp_file");
        const std::string covf = required_path(ini, "sptpol_TEEE_cov_file");
        const std::string wdir = required_path(ini, "sptpol_TEEE_window_dir");
        const std::string beamf = required_path(ini, "sptpol_TEEE_beam_file");
        auto dl = read_lines(desc);
        if (dl.size() < 2) fail(CMBL_ERR_FORMAT, "SPTpol: short desc file %s", desc.c_str());
        nbin = (int)field(dl[0], 0, desc);
        const int nfreq = (int)field(dl[0], 1, desc);
        lmin = (int)field(dl[1], 0, desc);
        lmax = (int)field(dl[1], 1, desc);
        if (nfreq != 1) fail(CMBL_ERR_FORMAT, "Sorry, current code wont work for multiple freqs");
        if (lmin < 2 || lmin >= lmax) fail(CMBL_ERR_FORMAT, "Invalid lranges for sptpol");
        if (nbin < 1) fail(CMBL_ERR_FORMAT, "SPTpol: nbin < 1");
        nband = 2;
        nall = 2 * nbin;
        nbeam = 2;   // N_BEAM_EXPECTED (:20)
        cl_lmax[0] = cl_lmax[4] = cl_lmax[5] = lmax + 1;     // (T,T) (E,T) (E,E)
        auto bl = read_lines(bpf);
        if ((int)bl.size() < 3 * nbin) fail(CMBL_ERR_FORMAT, "SPTpol: %s needs %d records", bpf.c_str(), 3 * nbin);
        std::vector<double> spec3(3 * nbin);
        for (int q = 0; q < 3 * nbin; q++) spec3[q] = field(bl[q], 1, bpf);   // spec(j,i): TE, EE, TT
        auto cov = read_direct_matrix(covf, nall);
        if (EEonly || TEonly) {   // :243-262
            for (int i = 0; i < nbin; i++)
                for (int j = nbin; j < 2 * nbin; j++) {
                    cov[(size_t)i * nall + j] *= 1e12;
                    cov[(size_t)j * nall + i] *= 1e12;
                }
            if (EEonly)
                for (int i = 0; i < nbin; i++)
                    for (int j = 0; j < nbin; j++) cov[(size_t)i * nall + j] *= 1e24;
            if (TEonly)
                for (int i = nbin; i < 2 * nbin; i++)
                    for (int j = nbin; j < 2 * nbin; j++) cov[(size_t)i * nall + j] *= 1e24;
        }
        const int NL = lmax - lmin + 1;
        std::vector<double> win((size_t)NL * nall);
        for (int i = 0; i < nall; i++) {        // window_<i>: "l value" records (:304-309)
            const std::string wf = wdir + "window_" + std::to_string(i + 1);
            auto wl = read_lines(wf);
            if ((int)wl.size() < NL) fail(CMBL_ERR_FORMAT, "SPTpol: %s needs %d records", wf.c_str(), NL);
            for (int l = 0; l < NL; l++) win[(size_t)l * nall + i] = field(wl[l], 1, wf);
        }
        auto be = read_lines(beamf);
        if ((int)be.size() < nbeam * nall) fail(CMBL_ERR_FORMAT, "SPTpol: %s needs %d records", beamf.c_str(), nbeam * nall);
        std::vector<double> beam((size_t)nbeam * nall);
        for (int q = 0; q < nbeam * nall; q++) beam[q] = field(be[q], 1, beamf);
        std::vector<double> spec(nall);
        for (int i = 0; i < nall; i++) spec[i] = spec3[i];   // TE then EE (:511-513)
        // per-l tables from l = lmin - 2, filled for lmin - 1 .. lmax + 1 (:202-211)
        std::vector<double> tab((size_t)(NL + 4) * 4, 0.0);
        for (int q = 1; q < NL + 3; q++) {
            const double l = (double)(lmin - 2 + q);
            const double conv = (l * (l + 1.0)) / SP_TWOPI;
            tab[(size_t)q * 4 + 0] = (l * l * l) / conv;
            tab[(size_t)q * 4 + 1] = conv;
            tab[(size_t)q * 4 + 2] = 0.5 / (l * l);
            tab[(size_t)q * 4 + 3] = std::log(l / 80.0);
        }
        int fields[3] = {1, 2, 0};   // TE, EE (Theory%ClArray(CL_T, CL_E), (CL_E, CL_E))
        finish(win, cov, spec, beam, tab, fields);
    }

    void read_bb(const Ini &ini) {             // SPTpol_BB_ReadIni / InitSPTpolBBData (:56-438)
        if (logical(ini, "sptpol_blind_r"))
            fail(CMBL_ERR_UNSUPPORTED, "sptpol_blind_r: the r blinding offset depends on CMB%%InitPower, "
                                       "which the batched likelihood does not receive");
        const bool blind_abb = logical(ini, "sptpol_blind_abb");
        const bool drop[3] = {logical(ini, "sptpol_drop_150x150ghz"), logical(ini, "sptpol_drop_90x150ghz"),
                              logical(ini, "sptpol_drop_90x90ghz")};
        if (drop[0] && drop[1] && drop[2]) fail(CMBL_ERR_FORMAT, "Error: SPTpol has no bandpowers left after drop flags");
        dev.pr_on[0] = logical(ini, "sptpol_cal_prior");
        dev.inv_cal[0] = real4(ini, "sptpol_invCal_90x90", 0.0004f);
        dev.inv_cal[1] = real4(ini, "sptpol_invCal_90x150", 0.0f);
        dev.inv_cal[2] = real4(ini, "sptpol_invCal_150x150", 0.0004f);
        dev.pr_on[1] = logical(ini, "sptpol_Add_prior");
        dev.pr_mean[1] = real4(ini, "sptpol_meanAdd", 0.0132f);
        dev.pr_sigma[1] = real4(ini, "sptpol_sigmaAdd", 0.0055f);
        nuisance_names = load_paramnames(required_path(ini, "sptpol_BB_params_file"), &n_nuis);
        if (n_nuis < 16)
            fail(CMBL_ERR_FORMAT, "SPTPOL_BB needs 16 nuisance parameters (Abb .. beam factors), got %d", n_nuis);
        if (logical(ini, "print_spectrum")) fail(CMBL_ERR_UNSUPPORTED, "SPTpol print_spectrum is not supported");
        const std::string desc = required_path(ini, "sptpol_BB_desc_file");
        const std::string bpf = required_path(ini, "sptpol_BB_bp_file");
        const std::string covf = required_path(ini, "sptpol_BB_cov_file");
        const std::string wfile = required_path(ini, "sptpol_BB_window_file");
        const std::string beamf = required_path(ini, "sptpol_BB_beam_file");
        auto dl = read_lines(desc);
        if (dl.size() < 2) fail(CMBL_ERR_FORMAT, "SPTpol: short desc file %s", desc.c_str());
        nbin = (int)field(dl[0], 0, desc);
        const int nfreq = (int)field(dl[0], 1, desc);
        lmin = (int)field(dl[1], 0, desc);
        lmax = (int)field(dl[1], 1, desc);
        if (nfreq != 2) fail(CMBL_ERR_FORMAT, "Sorry, current code assumes 95 and 150 GHz only");
        if ((int)dl.size() < 2 + nfreq) fail(CMBL_ERR_FORMAT, "SPTpol: %s lacks the effective frequencies", desc.c_str());
        const double eff[2] = {field(dl[2], 0, desc), field(dl[3], 0, desc)};
        if (lmin < 2 || lmin >= lmax) fail(CMBL_ERR_FORMAT, "Invalid lranges for sptpol");
        nband = 3;
        nall = 3 * nbin;
        cl_lmax[2 * 4 + 2] = lmax + 1;   // (B,B)
        const double pf[3][2] = {{eff[0], eff[0]}, {eff[0], eff[1]}, {eff[1], eff[1]}};   // effFreqs (:207-215)
        for (int k = 0; k < 3; k++) dev.dust_scale[k] = dust_scaling(pf[k][0], pf[k][1]);
        // bandpowers: records "lcen llo lhi bb90 bb90x150 bb150", comment records skipped (:232-253)
        std::vector<double> spec(nall);
        {
            auto bl = read_lines(bpf);
            int k = 0;
            for (auto &s0 : bl) {
                if (k >= nbin) break;
                const size_t a = s0.find_first_not_of(" \t\r");
                const std::string s = a == std::string::npos ? std::string() : s0.substr(a);
                const size_t h = s.find('#'), e = s.find('!');
                const int idx = (h == std::string::npos ? 0 : (int)h + 1) + (e == std::string::npos ? 0 : (int)e + 1);
                if (idx == 1) continue;
                spec[0 * nbin + k] = field(s, 5, bpf);
                spec[1 * nbin + k] = field(s, 4, bpf);
                spec[2 * nbin + k] = field(s, 3, bpf);
                k++;
            }
            if (k < nbin) fail(CMBL_ERR_FORMAT, "SPTpol: %s holds %d of %d bandpowers", bpf.c_str(), k, nbin);
        }
        auto cov = read_direct_matrix(covf, nall);
        for (int band = 0; band < 3; band++) {   // drop flags (:262-299)
            if (!drop[band]) continue;
            for (int i = 0; i < nbin; i++) {
                const int t = band * nbin + i;
                const double d = cov[(size_t)t * nall + t];
                for (int q = 0; q < nall; q++) cov[(size_t)t * nall + q] = cov[(size_t)q * nall + t] = 0.0;
                cov[(size_t)t * nall + t] = 1e12 * d;
            }
        }
        const int NL = lmax - lmin + 1;
        std::vector<double> win((size_t)NL * nall);
        {
            auto b = read_bytes(wfile);
            if (b.size() < 8 + (size_t)NL * nall * 8) fail(CMBL_ERR_FORMAT, "SPTpol: %s is too short", wfile.c_str());
            int32_t i0, i1;
            std::memcpy(&i0, b.data(), 4);
            std::memcpy(&i1, b.data() + 4, 4);
            if (i0 != lmin || i1 != lmax) fail(CMBL_ERR_FORMAT, "mismatched sptpol BB window ranges, quitting");
            const double *p = reinterpret_cast<const double *>(b.data() + 8);
            std::vector<double> cm((size_t)NL * nall);
            std::memcpy(cm.data(), p, cm.size() * 8);
            for (int i = 0; i < nall; i++)
                for (int l = 0; l < NL; l++) win[(size_t)l * nall + i] = cm[(size_t)i * NL + l];
        }
        std::vector<double> beam;
        {
            auto b = read_bytes(beamf);
            if (b.size() < 8) fail(CMBL_ERR_FORMAT, "SPTpol: %s is too short", beamf.c_str());
            int32_t neff, nt;
            std::memcpy(&neff, b.data(), 4);
            std::memcpy(&nt, b.data() + 4, 4);
            if (neff != nall) fail(CMBL_ERR_FORMAT, "SPTpol: mismatched beam error file claimed Nbandpowers");
            if (nt < 1 || nt > nbin) fail(CMBL_ERR_FORMAT, "SPTpol: invalid beam error file claimed Nbeam_terms");
            if (nt != 7) fail(CMBL_ERR_FORMAT, "SPTpol: expected  a different number of beam error terms.");
            if (b.size() < 8 + (size_t)nt * neff * 8) fail(CMBL_ERR_FORMAT, "SPTpol: %s is too short", beamf.c_str());
            nbeam = nt;
            beam.resize((size_t)nt * neff);
            std::memcpy(beam.data(), b.data() + 8, beam.size() * 8);
        }
        if (blind_abb) {
            const std::string f = required_path(ini, "sptpol_blind_abb_file");
            auto b = read_bytes(f);
            if (b.size() < 8) fail(CMBL_ERR_FORMAT, "SPTpol: %s is too short", f.c_str());
            std::memcpy(&dev.blind_abb, b.data(), 8);
        }
        std::vector<double> tensor(NL, 0.0);
        const std::string rt = ini.str("r_template_file");
        if (!rt.empty()) {   // records "l tt ee bb te" (:418-433)
            for (auto &s0 : read_lines(rt)) {
                const size_t a = s0.find_first_not_of(" \t\r");
                if (a == std::string::npos) continue;
                const std::string s = s0.substr(a);
                const size_t h = s.find('#'), e = s.find('!');
                const int idx = (h == std::string::npos ? 0 : (int)h + 1) + (e == std::string::npos ? 0 : (int)e + 1);
                if (idx == 1) continue;
                const int l = (int)field(s, 0, rt);
                if (l <= lmax && l >= lmin) tensor[l - lmin] = field(s, 3, rt);
            }
        }
        // per-l tables from l = lmin - 2, filled for lmin .. lmax (:222-228)
        std::vector<double> tab((size_t)(NL + 4) * 4, 0.0);
        for (int q = 2; q < NL + 2; q++) {
            const double l = (double)(lmin - 2 + q);
            tab[(size_t)q * 4 + 0] = (l * (l + 1.0)) / (double)(3000.0f * 3001.0f);
            tab[(size_t)q * 4 + 1] = ((l + 1.0) / 81.0) * std::pow(80.0 / l, (double)1.42f);
            tab[(size_t)q * 4 + 2] = tensor[q - 2];
        }
        int fields[3] = {5, 5, 5};   // BB (Theory%ClArray(CL_B, CL_B))
        finish(win, cov, spec, beam, tab, fields);
    }

    struct WsLayout { size_t part, add, total; };
    WsLayout layout(int W) const {
        auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
        WsLayout o{};
        o.part = al(qf.workspace_size(W));
        o.add = o.part + al((size_t)std::max(1, n_part_rows) * W * 8);
        o.total = o.add + al((size_t)W * 8);
        return o;
    }
    size_t workspace_size(int W) const override { return layout(W).total; }

    void loglike_batch(int W, const double *dl, long long ld_field, long long ld_walker, const double *nuis,
                       long long ld_nuis, double *out, void *ws, hipStream_t stream) override {
        if (W <= 0) return;
        if (!nuis) fail(CMBL_ERR_ARG, "%s needs its %d nuisance parameters", name.c_str(), n_nuis);
        if (ld_nuis < n_nuis && W > 1) fail(CMBL_ERR_ARG, "ld_nuis %lld < %d nuisance parameters", ld_nuis, n_nuis);
        if (ld_field < need_lmax + 1) fail(CMBL_ERR_ARG, "ld_field %lld < %d (l up to %d)", ld_field, need_lmax + 1, need_lmax);
        const int maxf = kind == SP_BB ? 5 : 2;
        if (W > 1 && ld_walker != 0 && ld_walker < (long long)(maxf + 1) * ld_field)
            fail(CMBL_ERR_ARG, "ld_walker must cover theory fields 0..%d", maxf);
        if (!ws) {
            own_ws.grow(workspace_size(W));
            ws = own_ws.p;
        }
        const WsLayout o = layout(W);
        char *base = static_cast<char *>(ws);
        double *partial = reinterpret_cast<double *>(base + o.part);
        double *addend = reinterpret_cast<double *>(base + o.add);
        const int tiles = (W + 63) / 64;
        const bool vec_ok = ((reinterpret_cast<uintptr_t>(dl) & 15) == 0) && ld_field % 2 == 0 && ld_walker % 2 == 0;
        if (dev.nitem > 0) {
            const int nblk = 8 * tiles * ((dev.nitem + 7) / 8);
            timed_launch("sptpol_window_kernel", stream, [&](hipEvent_t e0, hipEvent_t e1) {
#define SP_WINDOW(K, A)                                                                                        \
    hipExtLaunchKernelGGL(sptpol_window_kernel<K, A>, dim3(nblk), dim3(256), 0, stream, e0, e1, 0, dev, dl, ld_field, \
                          ld_walker, nuis, ld_nuis, partial, W, tiles, (int)vec_ok)
                if (kind == SP_BB) SP_WINDOW(SP_BB, false);
                else if (aberration) SP_WINDOW(SP_TEEE, true);
                else SP_WINDOW(SP_TEEE, false);
#undef SP_WINDOW
            });
            HIP_CHECK(hipGetLastError());
        }
        const dim3 dgrid((W + 63) / 64, (qf.Np + SP_DB - 1) / SP_DB);
        timed_launch("sptpol_delta_kernel", stream, [&](hipEvent_t e0, hipEvent_t e1) {
            if (kind == SP_BB)
                hipExtLaunchKernelGGL(sptpol_delta_kernel<SP_BB>, dgrid, dim3(64 * SP_DB), 0, stream, e0, e1, 0, dev,
                                      (const double *)partial, nuis, ld_nuis, qf.x_rows(ws), addend,
                                      qf.counters(ws, W), qf.n_counters(W), W);
            else
                hipExtLaunchKernelGGL(sptpol_delta_kernel<SP_TEEE>, dgrid, dim3(64 * SP_DB), 0, stream, e0, e1, 0, dev,
                                      (const double *)partial, nuis, ld_nuis, qf.x_rows(ws), addend,
                                      qf.counters(ws, W), qf.n_counters(W), W);
        });
        HIP_CHECK(hipGetLastError());
        qf.launch(W, ws, addend, out, stream, "sptpol_quadform");
    }
};

std::unique_ptr<Like> make_sptpol(const Ini &ini, const std::string &tag) {
    return std::unique_ptr<Like>(new SPTpol(ini, tag));
}

}  // namespace cmamd
