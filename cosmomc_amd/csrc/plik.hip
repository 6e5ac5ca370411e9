// Native plik_lite likelihood (reference TPlikLiteLikelihood, source/CMB.f90:30-329)
// batched over W walkers on MI355X (gfx950).
//
// Per walker:  cl_b  = sum_{l in bin b} D_l w_l          (CMB.f90:315-325)
//              Delta = X - cl / cal^2                    (CMB.f90:326)
//              -lnL  = Delta^T C^-1 Delta / 2            (CMB.f90:327, Matrix_QuadForm)
//
// Kernels (one launch each, same stream):
//   plik_bin_delta      one workgroup per walker: the walker's D_l rows are
//                       streamed once from HBM (coalesced) into LDS as D_l*w_l
//                       products, then every bin is a contiguous LDS sum.
//                       Writes Delta[w][Np] (Np = nused rounded up to 64).
//   plik_quadform_pairs C^-1 is split into 64x64 blocks; only the upper block
//                       triangle (I <= J) is visited (C^-1 symmetric), one
//                       workgroup per (block pair, 64-walker tile).  T =
//                       C_IJ Delta_J^T on the f64 MFMA (v_mfma_f64_16x16x4f64),
//                       then the column dot with Delta_I and x2 off-diagonal.
//                       Writes partial[pair][w].
//   plik_finalize       -lnL[w] = sum_pair partial[pair][w] / 2, fixed order.
#include <cmath>
#include <cstring>
#include <fstream>

#include "common.h"

namespace cmamd {

typedef double f64x4 __attribute__((ext_vector_type(4)));

static constexpr int TILE = 64;          // C^-1 block edge and walker tile
static constexpr int LDSW = TILE + 2;    // padded LDS row (66 doubles): conflict-free f64 MFMA fragments

// ------------------------------------------------------------------ kernels

struct BinInfo {
    int field;   // 0 TT, 1 TE, 2 EE  (Theory%Cls (1,1) (2,1) (2,2))
    int lmin;    // absolute l
    int lmax;
    int pad;
};

__global__ __launch_bounds__(256) void plik_bin_delta(
    const double *__restrict__ dl, long long ld_field, long long ld_walker,
    const double *__restrict__ nuis, long long ld_nuis,
    const double *__restrict__ wts,          // by absolute l
    const BinInfo *__restrict__ bins, const double *__restrict__ X,
    int nused, int Np, int3 flo, int3 fhi, int3 foff,
    double *__restrict__ delta)
{
    extern __shared__ double prod[];       // D_l * w_l for the used l ranges of each field
    const int w = blockIdx.x;
    const double *D = dl + (long long)w * ld_walker;
    const int lo[3] = {flo.x, flo.y, flo.z};
    const int hi[3] = {fhi.x, fhi.y, fhi.z};
    const int off[3] = {foff.x, foff.y, foff.z};
#pragma unroll
    for (int f = 0; f < 3; f++) {
        if (hi[f] < lo[f]) continue;
        const double *Df = D + f * ld_field;
        for (int l = lo[f] + (int)threadIdx.x; l <= hi[f]; l += blockDim.x)
            prod[off[f] + l - lo[f]] = Df[l] * wts[l];
    }
    __syncthreads();
    const double cal = nuis[(long long)w * ld_nuis];
    const double c2 = cal * cal;
    double *out = delta + (long long)w * Np;
    for (int i = threadIdx.x; i < Np; i += blockDim.x) {
        double d = 0.0;
        if (i < nused) {
            const BinInfo b = bins[i];
            const double *p = prod + off[b.field] - lo[b.field];
            double acc = 0.0;
            for (int l = b.lmin; l <= b.lmax; l++) acc += p[l];
            d = X[i] - acc / c2;
        }
        out[i] = d;
    }
}

__global__ __launch_bounds__(256) void plik_quadform_pairs(
    const double *__restrict__ invcov, int Np,
    const double *__restrict__ delta, int W, int Wpad,
    const int2 *__restrict__ pairs, double *__restrict__ partial)
{
    __shared__ __attribute__((aligned(16))) double smem[2 * TILE * LDSW];
    double *As = smem;                    // As[i][k] = C^-1[I*64+i][J*64+k]
    double *Bs = smem + TILE * LDSW;      // Bs[n][k] = Delta[w0+n][J*64+k]
    const int p = blockIdx.x;
    const int I = pairs[p].x, J = pairs[p].y;
    const int w0 = blockIdx.y * TILE;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

    for (int e = tid; e < TILE * TILE / 2; e += 256) {
        const int r = e >> 5, c2 = (e & 31) * 2;
        double2 a = *reinterpret_cast<const double2 *>(invcov + (size_t)(I * TILE + r) * Np + J * TILE + c2);
        *reinterpret_cast<double2 *>(As + r * LDSW + c2) = a;
        const int w = w0 + r;
        double2 b = make_double2(0.0, 0.0);
        if (w < W) b = *reinterpret_cast<const double2 *>(delta + (size_t)w * Np + J * TILE + c2);
        *reinterpret_cast<double2 *>(Bs + r * LDSW + c2) = b;
    }
    __syncthreads();

    const int li = lane & 15, lk = lane >> 4;
    f64x4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; t++) acc[t] = f64x4{0.0, 0.0, 0.0, 0.0};
    const double *brow = Bs + (16 * wave + li) * LDSW + lk;
#pragma unroll 4
    for (int kk = 0; kk < TILE / 4; kk++) {
        const double b = brow[4 * kk];
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const double a = As[(16 * t + li) * LDSW + 4 * kk + lk];
            acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[t], 0, 0, 0);
        }
    }
    __syncthreads();
    // Delta_I tile into the A buffer: As[n][i] = Delta[w0+n][I*64+i]
    for (int e = tid; e < TILE * TILE / 2; e += 256) {
        const int r = e >> 5, c2 = (e & 31) * 2;
        const int w = w0 + r;
        double2 v = make_double2(0.0, 0.0);
        if (w < W) v = *reinterpret_cast<const double2 *>(delta + (size_t)w * Np + I * TILE + c2);
        *reinterpret_cast<double2 *>(As + r * LDSW + c2) = v;
    }
    __syncthreads();
    // f64 16x16x4 C/D layout: col = lane&15 (walker n), row = (lane>>4) + 4*r (i)
    const int n = 16 * wave + li;
    double s = 0.0;
#pragma unroll
    for (int t = 0; t < 4; t++)
#pragma unroll
        for (int r = 0; r < 4; r++) s += acc[t][r] * As[n * LDSW + 16 * t + lk + 4 * r];
    s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    if (lk == 0 && w0 + n < W) partial[(size_t)p * Wpad + w0 + n] = (I == J ? s : 2.0 * s);
}

__global__ void plik_finalize(const double *__restrict__ partial, int npairs, int W, int Wpad,
                              double *__restrict__ out)
{
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= W) return;
    double s = 0.0;
    for (int p = 0; p < npairs; p++) s += partial[(size_t)p * Wpad + w];
    out[w] = s / 2.0;
}

// clik packing (cliklike.f90:138-163) -> D_l fields TT, TE, EE for the native kernel
__global__ void clik_to_dl(const double *__restrict__ clp, long long ld, int lmax_tt, int lmax_ee,
                           int lmax_bb, int lmax_te, double *__restrict__ dl, long long ld_field,
                           long long ld_walker, int lmax_out)
{
    const int w = blockIdx.y;
    const double *row = clp + (long long)w * ld;
    const long long o_tt = 0, o_ee = o_tt + lmax_tt + 1, o_bb = o_ee + lmax_ee + 1, o_te = o_bb + lmax_bb + 1;
    for (int l = blockIdx.x * blockDim.x + threadIdx.x; l <= lmax_out; l += gridDim.x * blockDim.x) {
        const double f = l >= 2 ? (double)l * (l + 1) / (2.0 * 3.14159265358979323846264338328) : 0.0;
        double *o = dl + (long long)w * ld_walker;
        o[l] = (l <= lmax_tt) ? row[o_tt + l] * f : 0.0;
        o[ld_field + l] = (l <= lmax_te) ? row[o_te + l] * f : 0.0;
        o[2 * ld_field + l] = (l <= lmax_ee) ? row[o_ee + l] * f : 0.0;
    }
}

// ------------------------------------------------------------------ host side

// Cholesky inverse of an SPD matrix (Matrix_Inverse: dpotrf 'L' + dpotri,
// source/Matrix_utils_new.f90:1478-1569), row-major, in place.
static void spd_inverse(std::vector<double> &A, int n) {
    for (int i = 0; i < n; i++)
        if (std::fabs(A[(size_t)i * n + i]) < 1e-30) fail(CMBL_ERR_NUMERIC, "Matrix_Inverse: very small diagonal");
    for (int j = 0; j < n; j++) {
        double d = A[(size_t)j * n + j];
        for (int k = 0; k < j; k++) d -= A[(size_t)j * n + k] * A[(size_t)j * n + k];
        if (!(d > 0.0)) fail(CMBL_ERR_NUMERIC, "Matrix_Inverse: covariance not positive definite (%d)", j + 1);
        d = std::sqrt(d);
        A[(size_t)j * n + j] = d;
        for (int i = j + 1; i < n; i++) {
            double s = A[(size_t)i * n + j];
            for (int k = 0; k < j; k++) s -= A[(size_t)i * n + k] * A[(size_t)j * n + k];
            A[(size_t)i * n + j] = s / d;
        }
    }
    for (int j = 0; j < n; j++) {           // L^-1, lower
        A[(size_t)j * n + j] = 1.0 / A[(size_t)j * n + j];
        for (int i = j + 1; i < n; i++) {
            double s = 0.0;
            for (int k = j; k < i; k++) s += A[(size_t)i * n + k] * A[(size_t)k * n + j];
            A[(size_t)i * n + j] = -s / A[(size_t)i * n + i];
        }
    }
    std::vector<double> T((size_t)n * n);
    for (int i = 0; i < n; i++)
        for (int j = 0; j <= i; j++) {
            double s = 0.0;
            for (int k = i; k < n; k++) s += A[(size_t)k * n + i] * A[(size_t)k * n + j];
            T[(size_t)i * n + j] = s;
            T[(size_t)j * n + i] = s;
        }
    A.swap(T);
}

static std::vector<double> flat(const std::vector<std::vector<double>> &m) {
    std::vector<double> v;
    for (auto &r : m) v.insert(v.end(), r.begin(), r.end());
    return v;
}

// Fortran unformatted sequential record holding an n x n column-major matrix
// (CMB.f90:236-245: read(lun) cov, then upper -> lower symmetrisation)
static std::vector<double> read_fortran_binary_matrix(const std::string &path, int n) {
    std::ifstream f(path, std::ios::binary);
    if (!f) fail(CMBL_ERR_IO, "cannot read %s", path.c_str());
    int32_t marker = 0;
    f.read(reinterpret_cast<char *>(&marker), 4);
    std::vector<double> colmajor((size_t)n * n);
    if ((size_t)marker != colmajor.size() * 8)
        fail(CMBL_ERR_FORMAT, "%s: record length %d != %d x %d doubles", path.c_str(), marker, n, n);
    f.read(reinterpret_cast<char *>(colmajor.data()), (std::streamsize)(colmajor.size() * 8));
    if (!f) fail(CMBL_ERR_FORMAT, "%s: short record", path.c_str());
    std::vector<double> rm((size_t)n * n);
    for (int i = 0; i < n; i++)            // cov(i,j) = colmajor[j*n+i]; keep upper (i<=j)
        for (int j = i; j < n; j++) {
            double v = colmajor[(size_t)j * n + i];
            rm[(size_t)i * n + j] = v;
            rm[(size_t)j * n + i] = v;
        }
    return rm;
}

std::string load_paramnames(const std::string &path, int *count) {
    std::ifstream f(path);
    if (!f) fail(CMBL_ERR_IO, "cannot read paramnames %s", path.c_str());
    std::string line, names;
    int n = 0;
    while (std::getline(f, line)) {
        auto t = split_ws(line);
        if (t.empty() || t[0][0] == '#') continue;
        std::string nm = t[0];
        if (!nm.empty() && nm.back() == '*') nm.pop_back();   // derived marker
        names += (n ? " " : "") + nm;
        n++;
    }
    *count = n;
    return names;
}

struct PlikLite final : Like {
    static constexpr int plmin = 30;     // CMB.f90:33
    static constexpr int nbins_total = 613;
    const int nbincl[3] = {215, 199, 199};
    int nused = 0, Np = 0, nblk = 0, npairs = 0, lmax_needed = 0;
    int flo[3], fhi[3], foff[3], lds_doubles = 0;
    DevBuf d_wts, d_bins, d_X, d_invcov, d_pairs;
    DevBuf conv;   // clik -> D_l staging

    explicit PlikLite(const Ini &ini) {
        tag = "PLIK_LITE";
        name = ini.str("name");
        if (name.empty()) {
            std::string fn = ini.filename();
            size_t s = fn.find_last_of('/');
            fn = fn.substr(s == std::string::npos ? 0 : s + 1);
            size_t d = fn.find_last_of('.');
            name = d == std::string::npos ? fn : fn.substr(0, d);
        }
        nuisance_names = load_paramnames(ini.relative_filename("calibration_param", true), &n_nuis);
        std::string use_cl = ini.str("use_cl");
        auto dat = load_txt(ini.relative_filename("data", true));
        auto blmin = flat(load_txt(ini.relative_filename("blmin", true)));
        auto blmax = flat(load_txt(ini.relative_filename("blmax", true)));
        auto wfile = flat(load_txt(ini.relative_filename("weights", true)));
        if ((int)dat.size() < nbins_total || dat[0].size() < 2)
            fail(CMBL_ERR_FORMAT, "plik_lite data file must have >= %d rows of >= 2 columns", nbins_total);
        int maxbin = nbincl[0];
        if ((int)blmin.size() < maxbin || (int)blmax.size() < maxbin)
            fail(CMBL_ERR_FORMAT, "plik_lite blmin/blmax need %d entries", maxbin);
        std::vector<int> bmin(maxbin), bmax(maxbin);
        for (int i = 0; i < maxbin; i++) {
            bmin[i] = (int)blmin[i] + plmin;   // CMB.f90:225-227
            bmax[i] = (int)blmax[i] + plmin;
        }
        const int nw = (int)wfile.size();
        lmax_needed = plmin + nw - 1;
        std::vector<double> wts(lmax_needed + 1, 0.0);
        for (int i = 0; i < nw; i++) {          // CMB.f90:230-233
            double ls = (double)(plmin + i);
            wts[plmin + i] = wfile[i] * (2.0 * 3.14159265358979323846264338328) / ls / (ls + 1.0);
        }
        std::vector<double> cov;
        std::string covb = ini.str("cov_file_binary");
        if (!covb.empty()) {
            cov = read_fortran_binary_matrix(ini.relative_filename("cov_file_binary", true), nbins_total);
        } else {
            cov = flat(load_txt(ini.relative_filename("cov_file", true)));
            if (cov.size() != (size_t)nbins_total * nbins_total)
                fail(CMBL_ERR_FORMAT, "plik_lite cov_file must be %d x %d", nbins_total, nbins_total);
        }
        // bins_for_L_range (CMB.f90:250-263)
        std::vector<int> usebins;
        bool ranged = false;
        std::string rng = ini.str("bins_for_L_range");
        if (!rng.empty()) {
            auto t = split_ws(rng);
            if (t.size() < 2) fail(CMBL_ERR_FORMAT, "bins_for_L_range needs two integers");
            int rmin = std::stoi(t[0]), rmax = std::stoi(t[1]);
            int mb = std::max(nbincl[0], std::max(nbincl[1], nbincl[2]));
            for (int i = 1; i <= mb; i++) {
                double c = (bmin[i - 1] + bmax[i - 1]) / 2.0;
                if (rmin <= c && c <= rmax) usebins.push_back(i);
            }
            ranged = true;
        }
        const char *names[3] = {"TT", "TE", "EE"};
        auto toks = split_ws(use_cl);
        std::vector<int> used_idx;
        std::vector<BinInfo> binfo;
        int offset = 0;
        for (int s = 0; s < 3; s++) {          // CMB.f90:265-297
            bool used = false;
            for (auto &t : toks) used |= (t == names[s]);
            if (used) {
                std::vector<int> bl;
                if (ranged) {
                    for (int b : usebins) if (b <= nbincl[s]) bl.push_back(b);
                } else {
                    for (int b = 1; b <= nbincl[s]; b++) bl.push_back(b);
                }
                int mx = 0;
                for (int b : bl) {
                    used_idx.push_back(b + offset - 1);
                    binfo.push_back({s, bmin[b - 1], bmax[b - 1], 0});
                    mx = std::max(mx, bmax[b - 1]);
                }
                const int ij[3][2] = {{1, 1}, {2, 1}, {2, 2}};
                cl_lmax[(ij[s][0] - 1) * 4 + (ij[s][1] - 1)] = mx;
            }
            offset += nbincl[s];
        }
        nused = (int)used_idx.size();
        if (nused == 0) fail(CMBL_ERR_FORMAT, "plik_lite: use_cl selects no bins");
        for (auto &b : binfo)
            if (b.lmin < plmin || b.lmax > lmax_needed) fail(CMBL_ERR_FORMAT, "plik_lite: bin outside weights range");
        std::vector<double> X(nused), ic((size_t)nused * nused);
        for (int i = 0; i < nused; i++) {       // CMB.f90:298-299
            X[i] = dat[used_idx[i]][1];
            for (int j = 0; j < nused; j++) ic[(size_t)i * nused + j] = cov[(size_t)used_idx[i] * nbins_total + used_idx[j]];
        }
        spd_inverse(ic, nused);                 // CMB.f90:300

        // device layout
        Np = (nused + TILE - 1) / TILE * TILE;
        nblk = Np / TILE;
        std::vector<double> icp((size_t)Np * Np, 0.0), Xp(Np, 0.0);
        for (int i = 0; i < nused; i++) {
            Xp[i] = X[i];
            for (int j = 0; j < nused; j++) icp[(size_t)i * Np + j] = ic[(size_t)i * nused + j];
        }
        std::vector<int2> pairs;
        for (int I = 0; I < nblk; I++)
            for (int J = I; J < nblk; J++) pairs.push_back(make_int2(I, J));
        npairs = (int)pairs.size();
        lds_doubles = 0;
        for (int f = 0; f < 3; f++) {
            flo[f] = 1 << 30;
            fhi[f] = -1;
        }
        for (auto &b : binfo) {
            flo[b.field] = std::min(flo[b.field], b.lmin);
            fhi[b.field] = std::max(fhi[b.field], b.lmax);
        }
        for (int f = 0; f < 3; f++) {
            foff[f] = lds_doubles;
            if (fhi[f] >= flo[f]) lds_doubles += fhi[f] - flo[f] + 1;
            else { flo[f] = 0; fhi[f] = -1; }
        }
        binfo.resize(Np, BinInfo{0, 1, 0, 0});
        d_wts.alloc(wts.size() * 8);
        d_wts.upload(wts.data(), wts.size() * 8);
        d_bins.alloc(binfo.size() * sizeof(BinInfo));
        d_bins.upload(binfo.data(), binfo.size() * sizeof(BinInfo));
        d_X.alloc(Xp.size() * 8);
        d_X.upload(Xp.data(), Xp.size() * 8);
        d_invcov.alloc(icp.size() * 8);
        d_invcov.upload(icp.data(), icp.size() * 8);
        d_pairs.alloc(pairs.size() * sizeof(int2));
        d_pairs.upload(pairs.data(), pairs.size() * sizeof(int2));
        const size_t lds = (size_t)lds_doubles * 8;
        if (lds > 64 * 1024)
            HIP_CHECK(hipFuncSetAttribute((const void *)plik_bin_delta,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    }

    static int wpad(int W) { return (W + TILE - 1) / TILE * TILE; }

    size_t workspace_size(int W) const override {
        const size_t Wp = (size_t)wpad(W);
        return (Wp * Np + (size_t)npairs * Wp) * sizeof(double);
    }

    void loglike_batch(int W, const double *dl, long long ld_field, long long ld_walker,
                       const double *nuis, long long ld_nuis, double *out, void *ws,
                       hipStream_t stream) override {
        if (W <= 0) return;
        if (n_nuis < 1 || !nuis) fail(CMBL_ERR_ARG, "plik_lite needs the calibration nuisance parameter");
        if (ld_field < lmax_needed + 1) fail(CMBL_ERR_ARG, "ld_field %lld < lmax+1 = %d", ld_field, lmax_needed + 1);
        if (ld_walker < 3 * ld_field) fail(CMBL_ERR_ARG, "ld_walker must cover the TT, TE, EE fields");
        const int Wp = wpad(W);
        if (!ws) {
            own_ws.grow(workspace_size(W));
            ws = own_ws.p;
        }
        double *delta = static_cast<double *>(ws);
        double *partial = delta + (size_t)Wp * Np;
        timed_launch("plik_bin_delta", stream, [&] {
            hipLaunchKernelGGL(plik_bin_delta, dim3(W), dim3(256), (size_t)lds_doubles * 8, stream, dl, ld_field,
                               ld_walker, nuis, ld_nuis, d_wts.as<double>(), d_bins.as<BinInfo>(), d_X.as<double>(),
                               nused, Np, make_int3(flo[0], flo[1], flo[2]), make_int3(fhi[0], fhi[1], fhi[2]),
                               make_int3(foff[0], foff[1], foff[2]), delta);
        });
        HIP_CHECK(hipGetLastError());
        timed_launch("plik_quadform_pairs", stream, [&] {
            hipLaunchKernelGGL(plik_quadform_pairs, dim3(npairs, Wp / TILE), dim3(256), 0, stream,
                               d_invcov.as<double>(), Np, delta, W, Wp, d_pairs.as<int2>(), partial);
        });
        HIP_CHECK(hipGetLastError());
        timed_launch("plik_finalize", stream, [&] {
            hipLaunchKernelGGL(plik_finalize, dim3((W + 255) / 256), dim3(256), 0, stream, partial, npairs, W, Wp,
                               out);
        });
        HIP_CHECK(hipGetLastError());
    }
};

std::unique_ptr<Like> make_plik_lite(const Ini &ini) { return std::unique_ptr<Like>(new PlikLite(ini)); }

// exported for the clik entry point (api.cpp)
void launch_clik_to_dl(const double *clp, long long ld, const int *lm, double *dl, long long ld_field,
                       long long ld_walker, int lmax_out, int W, hipStream_t stream) {
    hipLaunchKernelGGL(clik_to_dl, dim3((lmax_out + 256) / 256, W), dim3(256), 0, stream, clp, ld, lm[0], lm[1],
                       lm[2], lm[3], dl, ld_field, ld_walker, lmax_out);
    HIP_CHECK(hipGetLastError());
}

}  // namespace cmamd
