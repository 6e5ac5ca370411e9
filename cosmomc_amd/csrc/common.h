// Shared internals of libcosmomc_amd.so (not part of the C ABI).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/cosmomc_amd.h"

namespace cmamd {

// Error carrying a C-ABI code; caught at the ABI boundary (api.cpp).
struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

[[noreturn]] inline void fail(int code, const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    throw Error(code, buf);
}

#define HIP_CHECK(expr)                                                                      \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            ::cmamd::fail(CMBL_ERR_HIP, "%s:%d %s: %s", __FILE__, __LINE__, #expr,            \
                         hipGetErrorString(e_));                                             \
    } while (0)

// RAII device buffer
struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
    DevBuf() = default;
    explicit DevBuf(size_t n) { alloc(n); }
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    ~DevBuf() { release(); }
    void alloc(size_t n) {
        release();
        if (n) {
            HIP_CHECK(hipMalloc(&p, n));
            HIP_CHECK(hipMemset(p, 0, n));
        }
        bytes = n;
    }
    void grow(size_t n) {
        if (n > bytes) alloc(n);
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <class T> T *as() const { return static_cast<T *>(p); }
    void upload(const void *src, size_t n) { HIP_CHECK(hipMemcpy(p, src, n, hipMemcpyHostToDevice)); }
};

// ---------------- per-kernel event timing (cmbl_profile_*) ----------------
// Off by default.  When on, every library kernel launch is bracketed by a
// pair of HIP events recorded on the launch stream, so the average device
// duration of each kernel can be read back (bench.py roofline pass).
struct Profiler {
    bool on = false;
    struct Rec {
        hipEvent_t a, b;
    };
    std::map<std::string, std::vector<Rec>> pending;
    std::map<std::string, std::pair<double, long long>> done;   // total ms, count
    std::vector<hipEvent_t> pool;
    hipEvent_t get() {
        hipEvent_t e;
        if (!pool.empty()) {
            e = pool.back();
            pool.pop_back();
        } else {
            (void)hipEventCreate(&e);
        }
        return e;
    }
    void collect() {
        for (auto &kv : pending) {
            auto &d = done[kv.first];
            for (auto &r : kv.second) {
                float ms = 0.f;
                (void)hipEventSynchronize(r.b);
                (void)hipEventElapsedTime(&ms, r.a, r.b);
                d.first += ms;
                d.second += 1;
                pool.push_back(r.a);
                pool.push_back(r.b);
            }
            kv.second.clear();
        }
    }
};
Profiler &profiler();

// launch(start, stop) must pass the two events to hipExtLaunchKernelGGL, which
// stamps them from the kernel's own dispatch (the same interval rocprofv3
// reports), not from separate queue packets around it; null when profiling is off.
template <class F> inline void timed_launch(const char *name, hipStream_t stream, F &&launch) {
    Profiler &p = profiler();
    if (!p.on) {
        launch(hipEvent_t(nullptr), hipEvent_t(nullptr));
        return;
    }
    (void)stream;
    Profiler::Rec r{p.get(), p.get()};
    launch(r.a, r.b);
    p.pending[name].push_back(r);
    if (p.pending[name].size() > 4096) p.collect();
}

// ---------------- ini files (IniObjects.f90 subset) ----------------
// key = value lines, '#' comments, INCLUDE(file)/DEFAULT(file), first
// definition wins (TNameValueList ignoreDuplicates), overrides applied first
// (TIniFile%Override), relative file names resolved against the ini's
// directory (Ini_ReadRelativeFileName / ResolveLinkedFile, IniObjects.f90:403-424).
class Ini {
  public:
    void open(const std::string &filename);
    void override_text(const char *text);          // "key = value" lines
    bool has(const std::string &key) const { return kv_.count(key) != 0; }
    std::string str(const std::string &key, const std::string &def = "") const;
    std::string str_required(const std::string &key) const;
    std::string relative_filename(const std::string &key, bool required) const;
    std::string resolve_path(std::string value) const;     // the same rule for a value given directly
    const std::string &filename() const { return filename_; }

  private:
    void add_line(const std::string &line, bool only_if_undefined);
    void open_rec(const std::string &filename, bool only_if_undefined, int depth);
    std::map<std::string, std::string> kv_;
    std::string filename_;
};

std::string dirname_of(const std::string &path);
bool file_exists(const std::string &path);
// File%LoadTxt: whitespace-separated numeric matrix, '#' comment lines skipped
std::vector<std::vector<double>> load_txt(const std::string &path);
std::vector<std::string> split_ws(const std::string &s);
// .paramnames file -> space-separated names (derived '*' stripped), count
std::string load_paramnames(const std::string &path, int *count, std::string *derived = nullptr,
                            int *n_derived = nullptr);

struct PlikBinArgs;   // plikbin.h

// What a deferred quadratic-form launch (QuadForm::launch_deferred) leaves
// for the kernel that consumes it: -lnL of walker w is the fixed-order combine
// of quadform.h (qf_group_sum / qf_tree) over the partials of walker tile
// w / 64 at lane w % 64, + addend[w] when addend is not null.
struct QFDeferred {
    const double *partial = nullptr;   // [tiles][n_items][64]
    int n_items = 0;
    const double *addend = nullptr;
};

// A deferred quadratic form whose operand rows a later launch forms itself from
// a window pass's raw sums (the sampler's unified step launch, mh_step_kernel):
// Delta[w][k] = X[k] - S[w][k] / cal_w^2, every row calibrated.
struct QFItem;
struct QFSource {
    const double *Ct = nullptr;   // [Np][Np] C^-1 with halved diagonal blocks
    int Np = 0, xcd_map = 0;
    const QFItem *items = nullptr;
    int n_items = 0;
    double *partial = nullptr;    // [tiles][n_items][64]
    const double *X = nullptr;    // [Np] data vector, zero padded
    const double *delta = nullptr;   // [Wp][Np] the window stage's Delta rows (the in-launch-combine form)
    unsigned int *counters = nullptr;   // [tiles] split-K arrival tickets (zero between launches)
    int n_counters = 0;
};

// A small gaussian CMBlikes chi^2 (smallgauss.h) as one launch's arguments:
// its workgroups can run in cmbl_gauss_small_kernel or beside a deferred
// quadratic form's (QuadForm::launch_deferred, Like::corun_small).
struct SmallGaussDev {
    int nE, nX, has_corr, cal_index;
    double log_cal_prior;
    const int *e_to_x;                               // [nE] index into bigX or -1
    const double *e_main_const, *e_corr_const;       // [nE] fixed-spectrum window dots
    const double *fidcorr, *chat;                    // [nE]
    int ntask;
    const int *trow;                                 // [ntask][8] partial rows per task, -1 padded
    const int *e_main_t, *e_corr_t;                  // [nE + 1] task ranges per element
    const int *wcount;                               // live walkers [0, *wcount), or null: all
};
struct SmallGaussLaunch {
    SmallGaussDev d;
    const double *partial;   // [rows][W] window partial rows
    const double *nuis;      // [W][ld_nuis]
    long long ld_nuis;
    const double *M;         // [nX][nX] inverse covariance
    double *out;             // [W] -lnL
    int W;
    // the sampler's unified step launch (mh_step_kernel): partial holds the window
    // pass's raw sums, and a row r with row_cal[r] != 0 is divided by cal^2 (cal =
    // nuis[w * ld_nuis + stage_cal]) as it is loaded -- the operation the pass's
    // emit would have applied before storing it
    const unsigned char *row_cal;
    int stage_cal;
};

// Window stage of a likelihood: its first kernel contracts every walker's
// theory rows with fixed weights (plik_lite's binning, CMBlikes' bin windows).
// Exposed as columns, the stages of several likelihoods that read one theory
// buffer run as one pass over it (theorypass.hip), each walker's theory read
// once; each likelihood then runs its remaining kernels (after_window).
struct WinCol {
    int field, lo, hi;     // theory field (cmbl_loglike_batch order) and absolute l range
    const double *w;       // host: hi - lo + 1 weights
    int row;               // output row (CMBlikes partial row / plik bin)
    int cal;               // divide the sum by cal^2 (the stage's calibration parameter)
};
struct WinStage {
    int kind = 0;          // 0: out[row * W + w] (CMBlikes partial rows); 1: out[w * ld + row] = X[row] - sum (plik Delta)
    int cal_index = -1;    // calibration parameter in the likelihood's nuisance vector (-1: none)
    std::vector<WinCol> cols;
    const double *X = nullptr;   // kind 1: device data vector
    int ld = 0;                  // kind 1: Delta row stride
};

// ---------------- likelihood object ----------------
struct Like {
    virtual ~Like() = default;
    std::string name, tag, nuisance_names;
    int n_nuis = 0;
    // derived parameters (the '*' names of the nuisance paramnames,
    // DataLike%derivedParameters, GeneralTypes.f90:504-512, 658-664)
    std::string derived_names;
    int n_derived = 0;
    // (the base returns zeros, as TDataLikelihood_derivedParameters does)
    virtual void derived_batch(int W, const double *nuis, long long ld_nuis, double *out, long long ld_out,
                               hipStream_t stream) {
        (void)nuis, (void)ld_nuis;
        if (W <= 0 || n_derived <= 0) return;
        if (!out || ld_out < n_derived) fail(CMBL_ERR_ARG, "derived output needs %d columns", n_derived);
        HIP_CHECK(hipMemset2DAsync(out, (size_t)ld_out * 8, 0, (size_t)n_derived * 8, W, stream));
    }
    int speed = -1;
    int cl_lmax[16] = {0};
    std::string last_error;
    virtual size_t workspace_size(int W) const = 0;
    virtual void loglike_batch(int W, const double *dl, long long ld_field, long long ld_walker,
                               const double *nuis, long long ld_nuis, double *out, void *ws,
                               hipStream_t stream) = 0;
    // Sparse evaluation for the sampler's per-likelihood change mask: the same
    // launch over W walker slots, of which only [0, *wcount) (a device count)
    // are live; the caller has compacted the live walkers' inputs into those
    // slots.  Likelihoods without it are evaluated densely.
    virtual bool sparse_capable() const { return false; }
    virtual void loglike_batch_sparse(int W, const double *dl, long long ld_field, long long ld_walker,
                                      const double *nuis, long long ld_nuis, double *out, void *ws,
                                      hipStream_t stream, const int *wcount) {
        (void)W, (void)dl, (void)ld_field, (void)ld_walker, (void)nuis, (void)ld_nuis, (void)out, (void)ws;
        (void)stream, (void)wcount;
        fail(CMBL_ERR_UNSUPPORTED, "%s: no sparse evaluation", name.c_str());
    }
    // Deferred evaluation for the sampler's fast steps: the same launches as
    // loglike_batch except the quadratic form's split-K combine, which the
    // sampler's next mh_kernel performs (QFDeferred).  ws must stay untouched
    // until then.
    virtual bool deferred_capable() const { return false; }
    virtual QFDeferred loglike_batch_deferred(int W, const double *dl, long long ld_field, long long ld_walker,
                                              const double *nuis, long long ld_nuis, void *ws, hipStream_t stream) {
        (void)W, (void)dl, (void)ld_field, (void)ld_walker, (void)nuis, (void)ld_nuis, (void)ws, (void)stream;
        fail(CMBL_ERR_UNSUPPORTED, "%s: no deferred evaluation", name.c_str());
    }
    // Window stage (see WinStage): its columns, where the stage writes in ws,
    // and the likelihood's remaining kernels once a fused pass has run it.
    virtual bool window_stage(WinStage &st) const {
        (void)st;
        return false;
    }
    virtual double *window_out(void *ws, int W) const {
        (void)ws, (void)W;
        return nullptr;
    }
    // co: another likelihood's small chi^2 to run inside this one's deferred
    // quadratic-form launch (only with defer, only if accepts_corun())
    virtual QFDeferred after_window(int W, const double *nuis, long long ld_nuis, double *out, void *ws,
                                    hipStream_t stream, bool defer, const SmallGaussLaunch *co = nullptr) {
        (void)W, (void)nuis, (void)ld_nuis, (void)out, (void)ws, (void)stream, (void)defer, (void)co;
        fail(CMBL_ERR_UNSUPPORTED, "%s: no window stage", name.c_str());
    }
    virtual bool accepts_corun() const { return false; }
    // plik_lite's binning as a co-run body's arguments (plikbin.h) over theory
    // rows dl; false: not a plik_lite likelihood, or the layout does not fit
    virtual bool bin_args(PlikBinArgs &a, const double *dl, long long ld_field, long long ld_walker) const {
        (void)a, (void)dl, (void)ld_field, (void)ld_walker;
        return false;
    }
    // The deferred quadratic form after this likelihood's window stage as a
    // QFSource (its workspace ws for W walkers); false if it has none.
    virtual bool qf_source(QFSource &q, int W, void *ws) {
        (void)q, (void)W, (void)ws;
        return false;
    }
    // This likelihood's whole after-window stage as a small chi^2 another
    // launch can carry (same arguments as after_window); false if it has none.
    virtual bool corun_small(SmallGaussLaunch &a, int W, const double *nuis, long long ld_nuis, double *out,
                             void *ws) {
        (void)a, (void)W, (void)nuis, (void)ld_nuis, (void)out, (void)ws;
        return false;
    }
    // Move the l boundaries at which the window stage splits its dot products
    // to the given segment starts (absolute l, per theory field), so that
    // another likelihood's columns never straddle one; false if unsupported.
    virtual bool window_resegment(const std::map<int, std::vector<int>> &starts) {
        (void)starts;
        return false;
    }
    // The segmentation in force (opaque) and its restore, so a caller whose
    // resegment came to nothing can put the handle back as it found it.
    virtual std::map<int, std::vector<int>> window_segments() const { return {}; }
    virtual void window_set_segments(const std::map<int, std::vector<int>> &segs) { (void)segs; }
    // internal workspace for ws == nullptr
    DevBuf own_ws;
    // sticky CMBL_STATUS_* bits set by the kernels (cmbl_status)
    DevBuf status_buf;
    int *status_word() {
        if (!status_buf.p) status_buf.alloc(256);
        return status_buf.as<int>();
    }
};

// Doubles of one walker's theory the likelihood reads: fields in
// cmbl_loglike_batch order (TT, TE, EE, TB, EB, BB, PT, PE, PB, PP), each
// l = 0..cl_lmax of its pair; the last used field ends at its lmax.
inline long long theory_extent(const Like &L, long long ld_field) {
    static const int fi[10] = {1, 2, 2, 3, 3, 3, 4, 4, 4, 4}, fj[10] = {1, 1, 2, 1, 2, 3, 1, 2, 3, 4};
    long long ext = 0;
    for (int f = 0; f < 10; f++) {
        const int lm = L.cl_lmax[(fi[f] - 1) * 4 + (fj[f] - 1)];
        if (lm > 0) ext = std::max(ext, f * ld_field + lm + 1);
    }
    return ext;
}

std::unique_ptr<Like> make_plik_lite(const Ini &ini);
std::unique_ptr<Like> make_cmblikes(const Ini &ini, const std::string &tag);
std::unique_ptr<Like> make_sptpol(const Ini &ini, const std::string &tag);   // SPTPOL_TEEE / SPTPOL_BB

}  // namespace cmamd

struct cmbl {
    std::unique_ptr<cmamd::Like> like;
    // cmbl_loglike_batch_host: device buffers, pinned host staging and a stream
    // kept across calls, so a W = 1 call per evaluation (the Fortran LogLike
    // binding) allocates nothing; one host call at a time per handle
    std::mutex host_mu;
    cmamd::DevBuf h_dl, h_nuis, h_out, h_ws;
    void *pin = nullptr;
    size_t pin_bytes = 0;
    hipStream_t host_stream = nullptr;
    // cmbl_clik_compute_batch scratch when the caller passes no workspace: calls
    // that share it are serialised by clik_mu and ordered on the device by
    // clik_ev (recorded on the stream of the last call that used it)
    std::mutex clik_mu;
    cmamd::DevBuf clik_ws;
    hipEvent_t clik_ev = nullptr;
    ~cmbl() {
        if (clik_ev) {
            (void)hipEventSynchronize(clik_ev);
            (void)hipEventDestroy(clik_ev);
        }
        if (pin) (void)hipHostFree(pin);
        if (host_stream) (void)hipStreamDestroy(host_stream);
    }
};
