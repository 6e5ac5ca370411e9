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
//   quadform_ksplit     -lnL[w] = Delta^T C^-1 Delta / 2 on the f64 MFMA
//                       (quadform.hip: upper block triangle, split-K with an
//                       in-launch fixed-order reduction).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <functional>

#include "plikbin.h"
#include "quadform.h"

namespace cmamd {


// ------------------------------------------------------------------ kernels

// Binning + residual (plik_bin_body, plikbin.h): one workgroup per (walker,
// field).  Per-field blocks need at most 20 KB of LDS, so a W = 1024 launch
// (3072 blocks) runs in even rounds (one 51 KB block per walker: 768
// resident, a 1.33-round tail).  Block (0, 0) also zeroes the split-K arrival
// counters of the quadratic-form kernel that follows on the same stream, and
// the field-0 blocks the Delta padding.
__global__ __launch_bounds__(256) void plik_bin_delta(
    PlikBinArgs a, const double *__restrict__ nuis, long long ld_nuis,
    double *__restrict__ delta, unsigned int *__restrict__ counters, int n_counters,
    const int *__restrict__ wcount)   // sparse evaluation: walkers [0, *wcount) live (null: all)
{
    extern __shared__ __attribute__((aligned(16))) double prod[];
    const int w = blockIdx.x, f = blockIdx.y;
    const int tid = threadIdx.x;
    if (f == 0) {
        if (w == 0)
            for (int i = tid; i < n_counters; i += blockDim.x) counters[i] = 0u;
        double *out = delta + (long long)w * a.Np;
        for (int i = a.nused + tid; i < a.Np; i += blockDim.x) out[i] = 0.0;
    }
    if (wcount && w >= *wcount) return;
    plik_bin_body<false>(a, prod, w, f, nuis, ld_nuis, delta);
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

// ParamNames_Init (ObjectParamNames.f90:119-151): one name per non-empty line;
// a trailing '*' marks a derived parameter.  Returns the non-derived (MCMC)
// names -- the likelihood's DataParams, num_MCMC of them in *count -- and the
// derived ones (their DataLike%derivedParameters outputs) in *derived.
std::string load_paramnames(const std::string &path, int *count, std::string *derived, int *n_derived) {
    std::ifstream f(path);
    if (!f) fail(CMBL_ERR_IO, "cannot read paramnames %s", path.c_str());
    std::string line, names, dnames;
    int n = 0, nd = 0;
    while (std::getline(f, line)) {
        auto t = split_ws(line);
        if (t.empty() || t[0][0] == '#') continue;
        std::string nm = t[0];
        if (!nm.empty() && nm.back() == '*') {   // derived marker
            nm.pop_back();
            dnames += (nd ? " " : "") + nm;
            nd++;
            continue;
        }
        names += (n ? " " : "") + nm;
        n++;
    }
    *count = n;
    if (derived) *derived = dnames;
    if (n_derived) *n_derived = nd;
    return names;
}

struct PlikLite final : Like {
    static constexpr int plmin = 30;     // CMB.f90:33
    static constexpr int nbins_total = 613;
    const int nbincl[3] = {215, 199, 199};
    int nused = 0, Np = 0, lmax_needed = 0;
    FieldRanges fr{};
    int lds_doubles = 0;
    DevBuf d_wts, d_bins, d_X;
    std::vector<BinInfo> h_bins;   // the used bins (host), for the window stage
    std::vector<double> h_wts;     // weights by absolute l
    QuadForm qf;
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
        qf.init(ic, nused);
        Np = qf.Np;
        std::vector<double> Xp(Np, 0.0);
        for (int i = 0; i < nused; i++) Xp[i] = X[i];
        // LDS ranges per field, widened to even start / odd end for 16-byte access
        lds_doubles = 0;
        for (int f = 0; f < 3; f++) {
            fr.lo[f] = 1 << 30;
            fr.hi[f] = -1;
            fr.b0[f] = fr.b1[f] = 0;
        }
        for (size_t i = 0; i < binfo.size(); i++) {   // bins are in field order
            const auto &b = binfo[i];
            if (fr.hi[b.field] < 0) fr.b0[b.field] = (int)i;
            fr.b1[b.field] = (int)i + 1;
            fr.lo[b.field] = std::min(fr.lo[b.field], b.lmin);
            fr.hi[b.field] = std::max(fr.hi[b.field], b.lmax);
        }
        for (int f = 0; f < 3; f++) {
            if (fr.hi[f] >= fr.lo[f]) {
                fr.lo[f] &= ~1;
                fr.hi[f] |= 1;
                lds_doubles = std::max(lds_doubles, fr.hi[f] - fr.lo[f] + 1);
            } else {
                fr.lo[f] = 0;
                fr.hi[f] = -1;
            }
        }

        h_bins.assign(binfo.begin(), binfo.end());
        h_wts = wts;
        binfo.resize(Np, BinInfo{0, 1, 0, 0});
        int wmax = lmax_needed;
        for (int f = 0; f < 3; f++) wmax = std::max(wmax, fr.hi[f]);
        wts.resize((size_t)wmax + 2, 0.0);
        d_wts.alloc(wts.size() * 8);
        d_wts.upload(wts.data(), wts.size() * 8);
        d_bins.alloc(binfo.size() * sizeof(BinInfo));
        d_bins.upload(binfo.data(), binfo.size() * sizeof(BinInfo));
        d_X.alloc(Xp.size() * 8);
        d_X.upload(Xp.data(), Xp.size() * 8);
        const size_t lds = (size_t)lds_doubles * 8;
        if (lds > 64 * 1024)
            HIP_CHECK(hipFuncSetAttribute((const void *)plik_bin_delta,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    }

    size_t workspace_size(int W) const override { return qf.workspace_size(W); }

    void loglike_batch(int W, const double *dl, long long ld_field, long long ld_walker,
                       const double *nuis, long long ld_nuis, double *out, void *ws,
                       hipStream_t stream) override {
        run(W, dl, ld_field, ld_walker, nuis, ld_nuis, out, ws, stream, nullptr);
    }
    bool sparse_capable() const override { return true; }
    void loglike_batch_sparse(int W, const double *dl, long long ld_field, long long ld_walker, const double *nuis,
                              long long ld_nuis, double *out, void *ws, hipStream_t stream,
                              const int *wcount) override {
        run(W, dl, ld_field, ld_walker, nuis, ld_nuis, out, ws, stream, wcount);
    }

    bool deferred_capable() const override { return true; }

    PlikBinArgs bin_args_for(const double *dl, long long ld_field, long long ld_walker) const {
        PlikBinArgs a;
        a.dl = dl;
        a.ld_field = ld_field;
        a.ld_walker = ld_walker;
        a.wts = d_wts.as<double>();
        a.bins = d_bins.as<BinInfo>();
        a.X = d_X.as<double>();
        a.nused = nused;
        a.Np = Np;
        a.fr = fr;
        // 16-byte D_l loads need 16-byte aligned rows and the widened ranges inside each row
        a.vec_ok = ((reinterpret_cast<uintptr_t>(dl) & 15) == 0) && (ld_field % 2 == 0) && (ld_walker % 2 == 0);
        for (int f = 0; f < 3; f++)
            if (fr.hi[f] >= fr.lo[f] && fr.hi[f] >= ld_field) a.vec_ok = 0;
        a.lds_doubles = lds_doubles;
        return a;
    }
    bool bin_args(PlikBinArgs &a, const double *dl, long long ld_field, long long ld_walker) const override {
        if (ld_field < lmax_needed + 1 || (ld_walker != 0 && ld_walker < 3 * ld_field)) return false;
        a = bin_args_for(dl, ld_field, ld_walker);
        return true;
    }

    // window stage: bin i = sum_{l in bin} D_l w_l of field TT / TE / EE, then
    // Delta_i = X_i - bin_i / cal^2 (CMB.f90:315-326), in the quadratic form's rows
    bool window_stage(WinStage &st) const override {
        st.kind = 1;
        st.cal_index = 0;
        st.X = d_X.as<double>();
        st.ld = Np;
        st.cols.clear();
        for (size_t i = 0; i < h_bins.size(); i++) {
            const BinInfo &b = h_bins[i];
            st.cols.push_back(WinCol{b.field, b.lmin, b.lmax, h_wts.data() + b.lmin, (int)i, 1});
        }
        return true;
    }
    double *window_out(void *ws, int W) const override {
        (void)W;
        return qf.x_rows(ws);
    }
    bool accepts_corun() const override { return true; }
    bool qf_source(QFSource &q, int W, void *ws) override {
        if (W <= 0 || !ws) return false;
        q = qf.source(W, ws, d_X.as<double>());
        return true;
    }
    QFDeferred after_window(int W, const double *nuis, long long ld_nuis, double *out, void *ws, hipStream_t stream,
                            bool defer, const SmallGaussLaunch *co = nullptr) override {
        (void)nuis, (void)ld_nuis;
        if (co && !defer) fail(CMBL_ERR_ARG, "internal: a co-run needs the deferred quadratic form");
        if (W <= 0) return QFDeferred{};
        if (defer) return qf.launch_deferred(W, ws, nullptr, stream, "plik_quadform_ksplit", co, "plik_quadform_corun");
        HIP_CHECK(hipMemsetAsync(qf.counters(ws, W), 0, (size_t)qf.n_counters(W) * 4, stream));
        qf.launch(W, ws, nullptr, out, stream, "plik_quadform_ksplit");
        return QFDeferred{};
    }
    QFDeferred loglike_batch_deferred(int W, const double *dl, long long ld_field, long long ld_walker,
                                      const double *nuis, long long ld_nuis, void *ws, hipStream_t stream) override {
        if (!ws) fail(CMBL_ERR_ARG, "deferred evaluation needs a caller workspace");
        return run(W, dl, ld_field, ld_walker, nuis, ld_nuis, nullptr, ws, stream, nullptr, true);
    }

    QFDeferred run(int W, const double *dl, long long ld_field, long long ld_walker, const double *nuis,
                   long long ld_nuis, double *out, void *ws, hipStream_t stream, const int *wcount,
                   bool defer = false) {
        if (W <= 0) return QFDeferred{};
        if (n_nuis < 1 || !nuis) fail(CMBL_ERR_ARG, "plik_lite needs the calibration nuisance parameter");
        if (ld_field < lmax_needed + 1) fail(CMBL_ERR_ARG, "ld_field %lld < lmax+1 = %d", ld_field, lmax_needed + 1);
        // ld_walker == 0: every walker reads the same theory (a shared slow point)
        if (ld_walker != 0 && ld_walker < 3 * ld_field) fail(CMBL_ERR_ARG, "ld_walker must cover the TT, TE, EE fields");
        if (!ws) {
            own_ws.grow(workspace_size(W));
            ws = own_ws.p;
        }
        double *delta = qf.x_rows(ws);
        unsigned int *counters = qf.counters(ws, W);
        const PlikBinArgs a = bin_args_for(dl, ld_field, ld_walker);
        timed_launch("plik_bin_delta", stream, [&](hipEvent_t e0, hipEvent_t e1) {
            hipExtLaunchKernelGGL(plik_bin_delta, dim3(W, 3), dim3(256), (size_t)lds_doubles * 8, stream, e0, e1, 0, a,
                                  nuis, ld_nuis, delta, counters, qf.n_counters(W), wcount);
        });
        HIP_CHECK(hipGetLastError());
        if (defer) return qf.launch_deferred(W, ws, nullptr, stream, "plik_quadform_ksplit");
        qf.launch(W, ws, nullptr, out, stream, "plik_quadform_ksplit", wcount);
        return QFDeferred{};
    }
};

std::unique_ptr<Like> make_plik_lite(const Ini &ini) { return std::unique_ptr<Like>(new PlikLite(ini)); }

// exported for the clik entry point (api.cpp)
__global__ void negate_kernel(const double *in, double *out, int W)
{
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w < W) out[w] = -in[w];
}

void launch_negate(const double *in, double *out, int W, hipStream_t stream) {
    hipLaunchKernelGGL(negate_kernel, dim3((W + 255) / 256), dim3(256), 0, stream, in, out, W);
    HIP_CHECK(hipGetLastError());
}

void launch_clik_to_dl(const double *clp, long long ld, const int *lm, double *dl, long long ld_field,
                       long long ld_walker, int lmax_out, int W, hipStream_t stream) {
    hipLaunchKernelGGL(clik_to_dl, dim3((lmax_out + 256) / 256, W), dim3(256), 0, stream, clp, ld, lm[0], lm[1],
                       lm[2], lm[3], dl, ld_field, ld_walker, lmax_out);
    HIP_CHECK(hipGetLastError());
}

}  // namespace cmamd
