// C ABI of libcosmomc_amd.so (include/cosmomc_amd.h).  Every entry point
// catches internal errors and turns them into codes + messages.
#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <cstring>

#include "sampler.h"

namespace cmamd {
void sampler_create(cmbs *s, const cmbs_config_t *cfg);
void sampler_set_covariance(cmbs *s, const double *cov);
void sampler_set_test_gaussian(cmbs *s, const double *cov, const double *center);
void sampler_add_likelihood(cmbs *s, cmbl_t *like, const int *nuisance_indices, const double *dl, long long ld_field,
                            long long ld_walker);
void sampler_set_start(cmbs *s, const double *P0, hipStream_t stream);
void sampler_step(cmbs *s, int n_steps, int fast_only, hipStream_t stream);
void sampler_enable_history(cmbs *s, int capacity);
void sampler_history_stats(cmbs *s, int first, int last, double *means, double *covs, hipStream_t stream);
void sampler_get_state_host(cmbs *s, double *P, double *cur_like, double *mult, int *num_accept);
size_t sampler_state_bytes(const cmbs *s);
void sampler_history_restore(cmbs *s, int first, int count, const double *in, const double *terms);
void sampler_history_terms_host(cmbs *s, int first, int count, double *out);
void sampler_save_state(cmbs *s, void *buf, size_t bytes);
void sampler_load_state(cmbs *s, const void *buf, size_t bytes);
void launch_negate(const double *in, double *out, int W, hipStream_t stream);
void launch_clik_to_dl(const double *clp, long long ld, const int *lm, double *dl, long long ld_field,
                       long long ld_walker, int lmax_out, int W, hipStream_t stream);
}  // namespace cmamd

using cmamd::Error;

static void put_err(char *buf, size_t len, const char *msg) {
    if (buf && len) {
        std::strncpy(buf, msg, len - 1);
        buf[len - 1] = 0;
    }
}

template <class F> static int guarded(std::string *err, F &&f) {
    try {
        f();
        return CMBL_OK;
    } catch (const Error &e) {
        if (err) *err = e.what();
        return e.code;
    } catch (const std::exception &e) {
        if (err) *err = e.what();
        return CMBL_ERR_FORMAT;
    }
}

cmamd::Profiler &cmamd::profiler() {
    static Profiler p;
    return p;
}

extern "C" {

void cmbl_profile_enable(int on) {
    auto &p = cmamd::profiler();
    if (!on) p.collect();
    p.on = on != 0;
}

void cmbl_profile_reset(void) {
    auto &p = cmamd::profiler();
    p.collect();
    p.done.clear();
}

int cmbl_profile_read(const char *kernel, double *total_ms, long long *count) {
    auto &p = cmamd::profiler();
    p.collect();
    auto it = p.done.find(kernel ? kernel : "");
    if (it == p.done.end()) {
        if (total_ms) *total_ms = 0;
        if (count) *count = 0;
        return CMBL_ERR_ARG;
    }
    if (total_ms) *total_ms = it->second.first;
    if (count) *count = it->second.second;
    return CMBL_OK;
}

int cmbl_open(const char *tag, const char *dataset_path, const char *override_ini, cmbl_t **out, char *errbuf,
              size_t errlen) {
    std::string err;
    if (!out || !dataset_path || !tag) {
        put_err(errbuf, errlen, "cmbl_open: null argument");
        return CMBL_ERR_ARG;
    }
    *out = nullptr;
    int rc = guarded(&err, [&] {
        cmamd::Ini ini;
        ini.open(dataset_path);
        ini.override_text(override_ini);
        std::unique_ptr<cmbl_t> h(new cmbl_t);
        std::string t(tag);
        // tag -> likelihood class as CMBLikelihood_Add (source/CMB.f90:80-97)
        if (t == "PLIK_LITE") h->like = cmamd::make_plik_lite(ini);
        else if (t == "SPTPOL_TEEE" || t == "SPTPOL_BB") h->like = cmamd::make_sptpol(ini, t);   // CMB.f90:86-91
        else if (t == "WMAP")   // CMB.f90:75-84: needs the external WMAP likelihood library
            cmamd::fail(CMBL_ERR_UNSUPPORTED, "cmbl_open: dataset tag '%s' not supported", tag);
        else h->like = cmamd::make_cmblikes(ini, t);      // TCMBLikes, TBK_planck (BKPLANCK), TSmica_planck (SMICA)
        *out = h.release();
    });
    if (rc) put_err(errbuf, errlen, err.c_str());
    return rc;
}

void cmbl_close(cmbl_t *h) { delete h; }

const char *cmbl_last_error(const cmbl_t *h) { return h && h->like ? h->like->last_error.c_str() : ""; }

int cmbl_info(const cmbl_t *h, int *n_nuis, int *cl_lmax, int *speed, const char **name,
              const char **nuisance_names) {
    if (!h || !h->like) return CMBL_ERR_ARG;
    const auto &L = *h->like;
    if (n_nuis) *n_nuis = L.n_nuis;
    if (cl_lmax) std::memcpy(cl_lmax, L.cl_lmax, sizeof L.cl_lmax);
    if (speed) *speed = L.speed;
    if (name) *name = L.name.c_str();
    if (nuisance_names) *nuisance_names = L.nuisance_names.c_str();
    return CMBL_OK;
}

int cmbl_derived_info(const cmbl_t *h, int *n_derived, const char **derived_names) {
    if (!h || !h->like) return CMBL_ERR_ARG;
    if (n_derived) *n_derived = h->like->n_derived;
    if (derived_names) *derived_names = h->like->derived_names.c_str();
    return CMBL_OK;
}

int cmbl_derived_batch(cmbl_t *h, int W, const double *nuis, long long ld_nuis, double *derived, long long ld_derived,
                       void *stream) {
    if (!h || !h->like) return CMBL_ERR_ARG;
    return guarded(&h->like->last_error, [&] {
        if (W < 0) cmamd::fail(CMBL_ERR_ARG, "cmbl_derived_batch: bad arguments");
        h->like->derived_batch(W, nuis, ld_nuis, derived, ld_derived, (hipStream_t)stream);
    });
}

size_t cmbl_workspace_size(const cmbl_t *h, int W) { return h && h->like ? h->like->workspace_size(W) : 0; }

int cmbl_loglike_batch(cmbl_t *h, int W, const double *dl, long long ld_field, long long ld_walker,
                       const double *nuis, long long ld_nuis, double *out, void *workspace, void *stream) {
    if (!h || !h->like) return CMBL_ERR_ARG;
    return guarded(&h->like->last_error, [&] {
        if (W < 0 || (W > 0 && (!dl || !out))) cmamd::fail(CMBL_ERR_ARG, "cmbl_loglike_batch: bad arguments");
        h->like->loglike_batch(W, dl, ld_field, ld_walker, nuis, ld_nuis, out, workspace, (hipStream_t)stream);
    });
}


int cmbl_loglike_batch_host(cmbl_t *h, int W, const double *dl, long long ld_field, long long ld_walker,
                            const double *nuis, long long ld_nuis, double *out) {
    if (!h || !h->like) return CMBL_ERR_ARG;
    return guarded(&h->like->last_error, [&] {
        if (W <= 0) return;
        if (!dl || !out) cmamd::fail(CMBL_ERR_ARG, "cmbl_loglike_batch_host: bad arguments");
        std::lock_guard<std::mutex> lock(h->host_mu);
        const auto &L = *h->like;
        const size_t nd = (size_t)((W - 1) * ld_walker + cmamd::theory_extent(L, ld_field));
        const size_t nn = nuis ? (size_t)((W - 1) * ld_nuis + L.n_nuis) : 0;
        if (!h->host_stream) HIP_CHECK(hipStreamCreateWithFlags(&h->host_stream, hipStreamNonBlocking));
        const size_t pin_need = (nd + nn + (size_t)W) * 8;
        if (pin_need > h->pin_bytes) {
            if (h->pin) HIP_CHECK(hipHostFree(h->pin));
            h->pin = nullptr;
            HIP_CHECK(hipHostMalloc(&h->pin, pin_need, hipHostMallocDefault));
            h->pin_bytes = pin_need;
        }
        h->h_dl.grow(nd * 8);
        h->h_nuis.grow(std::max<size_t>(nn, 1) * 8);
        h->h_out.grow((size_t)W * 8);
        h->h_ws.grow(L.workspace_size(W));
        double *pdl = static_cast<double *>(h->pin), *pn = pdl + nd, *pout = pn + nn;
        std::memcpy(pdl, dl, nd * 8);                          // pinned staging: one DMA each way
        if (nn) std::memcpy(pn, nuis, nn * 8);
        hipStream_t st = h->host_stream;
        HIP_CHECK(hipMemcpyAsync(h->h_dl.p, pdl, nd * 8, hipMemcpyHostToDevice, st));
        if (nn) HIP_CHECK(hipMemcpyAsync(h->h_nuis.p, pn, nn * 8, hipMemcpyHostToDevice, st));
        h->like->loglike_batch(W, h->h_dl.as<double>(), ld_field, ld_walker, nn ? h->h_nuis.as<double>() : nullptr,
                               ld_nuis, h->h_out.as<double>(), h->h_ws.p, st);
        HIP_CHECK(hipMemcpyAsync(pout, h->h_out.p, (size_t)W * 8, hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipStreamSynchronize(st));
        std::memcpy(out, pout, (size_t)W * 8);
        int flags = 0;
        if (h->like->status_buf.p) {
            HIP_CHECK(hipMemcpy(&flags, h->like->status_buf.p, sizeof flags, hipMemcpyDeviceToHost));
            if (flags) {
                HIP_CHECK(hipMemset(h->like->status_buf.p, 0, sizeof flags));
                cmamd::fail(CMBL_ERR_NUMERIC, "%s: HL eigensolve did not converge (status %d)", L.name.c_str(), flags);
            }
        }
    });
}

int cmbl_status(cmbl_t *h, int *flags, int clear) {
    if (!h || !h->like || !flags) return CMBL_ERR_ARG;
    return guarded(&h->like->last_error, [&] {
        *flags = 0;
        if (!h->like->status_buf.p) return;
        HIP_CHECK(hipDeviceSynchronize());
        HIP_CHECK(hipMemcpy(flags, h->like->status_buf.p, sizeof(int), hipMemcpyDeviceToHost));
        if (clear && *flags) HIP_CHECK(hipMemset(h->like->status_buf.p, 0, sizeof(int)));
    });
}

// clik layout -> D_l rows + the native likelihood's scratch, carved from one workspace
struct ClikWs {
    int lm[6];
    long long ncl, ldf, ldw;
    int lmax_out;
    size_t bytes;
};

static ClikWs clik_ws_layout(const cmamd::Like &L, int W, const int *clik_lmax) {
    ClikWs c{};
    c.ncl = 0;
    for (int i = 0; i < 6; i++) {
        c.lm[i] = clik_lmax ? clik_lmax[i] : 0;
        c.ncl += c.lm[i] + 1;                // lmax = -1 -> absent (0 entries)
    }
    // D_l rows long enough for every spectrum the native likelihood reads
    c.lmax_out = std::max(L.cl_lmax[0], std::max(L.cl_lmax[4], L.cl_lmax[5]));
    c.ldf = c.lmax_out + 1;
    c.ldw = 3 * c.ldf;
    c.bytes = (size_t)c.ldw * W * 8 + (size_t)W * 8 + L.workspace_size(W);
    return c;
}

size_t cmbl_clik_workspace_size(const cmbl_t *h, int W) {
    return h && h->like && W > 0 ? clik_ws_layout(*h->like, W, nullptr).bytes : 0;
}

int cmbl_clik_compute_batch(cmbl_t *h, int W, const int *clik_lmax, const double *cl_and_pars, long long ld,
                            double *lnlike, void *workspace, void *stream) {
    if (!h || !h->like) return CMBL_ERR_ARG;
    return guarded(&h->like->last_error, [&] {
        if (h->like->tag != "PLIK_LITE") cmamd::fail(CMBL_ERR_UNSUPPORTED, "clik entry only routes to PLIK_LITE");
        if (W <= 0) return;
        if (!clik_lmax || !cl_and_pars || !lnlike) cmamd::fail(CMBL_ERR_ARG, "cmbl_clik_compute_batch: bad arguments");
        const ClikWs c = clik_ws_layout(*h->like, W, clik_lmax);
        const hipStream_t st = (hipStream_t)stream;
        auto run = [&](void *ws) {
            double *dl = static_cast<double *>(ws);
            double *mlnl = dl + (size_t)c.ldw * W;
            void *lws = mlnl + W;
            cmamd::launch_clik_to_dl(cl_and_pars, ld, c.lm, dl, c.ldf, c.ldw, c.lmax_out, W, st);
            // nuisance parameters follow the C_l blocks (cliklike.f90:157-163)
            h->like->loglike_batch(W, dl, c.ldf, c.ldw, cl_and_pars + c.ncl, ld, mlnl, lws, st);
            // lnlike = -(-lnL): clik_compute returns +lnL (cliklike.f90:166), negated on device
            cmamd::launch_negate(mlnl, lnlike, W, st);
        };
        if (workspace) {
            run(workspace);
            return;
        }
        // the handle's scratch: one host call at a time, and on the device after
        // every earlier call's kernels on whatever stream they ran
        std::lock_guard<std::mutex> lock(h->clik_mu);
        if (h->clik_ev) {
            if (h->clik_ws.bytes < c.bytes) HIP_CHECK(hipEventSynchronize(h->clik_ev));   // grow frees it
            HIP_CHECK(hipStreamWaitEvent(st, h->clik_ev, 0));
        } else {
            HIP_CHECK(hipEventCreateWithFlags(&h->clik_ev, hipEventDisableTiming));
        }
        h->clik_ws.grow(c.bytes);
        run(h->clik_ws.p);
        HIP_CHECK(hipEventRecord(h->clik_ev, st));
    });
}

// ------------------------------------------------------------ sampler

void cmbs_walker_seed(int seed_ij, int seed_kl, int walker, int *ij, int *kl) {
    // walker 0 keeps (seed_ij, seed_kl) -- the reference's rand_seed chain --
    // later walkers step ij through its full range, then kl.
    const long long t = (long long)seed_ij + walker;
    *ij = (int)(t % 31329);
    *kl = (int)(((long long)seed_kl + t / 31329) % 30082);
}

int cmbs_create(const cmbs_config_t *cfg, cmbs_t **out, char *errbuf, size_t errlen) {
    std::string err;
    if (!cfg || !out) return CMBL_ERR_ARG;
    *out = nullptr;
    std::unique_ptr<cmbs> s(new cmbs);
    if (const char *e = std::getenv("CMAMD_PIPE")) {   // fast-step schedule for A/B runs (cmamd_debug_pipeline)
        const int m = std::atoi(e);
        if (m == 0 || m == 3) s->pipe_mode = m;
        else   // modes 1, 2 and 4 were deleted in round 5: say so rather than run the default unannounced
            std::fprintf(stderr, "cosmomc_amd: CMAMD_PIPE=%s ignored (accepted: 0 unpipelined, 3 unified)\n", e);
    }
    if (const char *e = std::getenv("CMAMD_FOLD_G")) s->fold_g = std::atoi(e) != 0;   // A/B runs
    if (const char *e = std::getenv("CMAMD_QF_AHEAD")) s->qf_ahead = std::atoi(e) != 0;
    if (const char *e = std::getenv("CMAMD_FOLD_LATE_PRIO")) s->fold_late_prio = std::atoi(e) != 0;
    if (const char *e = std::getenv("CMAMD_QF_PRIO")) s->qf_prio = std::atoi(e) != 0;
    if (const char *e = std::getenv("CMAMD_FOLD_TPF")) s->fold_tpf = std::atoi(e) == 2 ? 2 : 1;
    int rc = guarded(&err, [&] { cmamd::sampler_create(s.get(), cfg); });
    if (rc) {
        put_err(errbuf, errlen, err.c_str());
        return rc;
    }
    *out = s.release();
    return CMBL_OK;
}

void cmbs_destroy(cmbs_t *s) { delete s; }
const char *cmbs_last_error(const cmbs_t *s) { return s ? s->last_error.c_str() : ""; }

int cmbs_set_covariance(cmbs_t *s, const double *cov) {
    if (!s || !cov) return CMBL_ERR_ARG;
    return guarded(&s->last_error, [&] { cmamd::sampler_set_covariance(s, cov); });
}

int cmbs_set_test_gaussian(cmbs_t *s, const double *cov, const double *center) {
    if (!s || !cov || !center) return CMBL_ERR_ARG;
    return guarded(&s->last_error, [&] { cmamd::sampler_set_test_gaussian(s, cov, center); });
}

int cmbs_add_likelihood(cmbs_t *s, cmbl_t *like, const int *nuisance_indices, const double *dl, long long ld_field,
                        long long ld_walker) {
    if (!s) return CMBL_ERR_ARG;
    return guarded(&s->last_error, [&] {
        cmamd::sampler_add_likelihood(s, like, nuisance_indices, dl, ld_field, ld_walker);
    });
}

int cmbs_set_start(cmbs_t *s, const double *P0, void *stream) {
    if (!s || !P0) return CMBL_ERR_ARG;
    return guarded(&s->last_error, [&] { cmamd::sampler_set_start(s, P0, (hipStream_t)stream); });
}

int cmbs_step(cmbs_t *s, int n_steps, int fast_only, void *stream) {
    if (!s) return CMBL_ERR_ARG;
    return guarded(&s->last_error, [&] { cmamd::sampler_step(s, n_steps, fast_only, (hipStream_t)stream); });
}

int cmbs_chain_moments(cmbs_t *s, int first, int last, const double *gmean, double *out, void *stream) {
    if (!s || !out) return CMBL_ERR_ARG;
    return guarded(&s->last_error,
                   [&] { cmamd::sampler_chain_moments(s, first, last, gmean, out, (hipStream_t)stream); });
}

int cmbs_set_trial_theory(cmbs_t *s, int like_index, double *dl_end, long long ld_field, long long ld_walker) {
    if (!s || !dl_end) return CMBL_ERR_ARG;
    return guarded(&s->last_error,
                   [&] { cmamd::sampler_set_trial_theory(s, like_index, dl_end, ld_field, ld_walker); });
}

int cmbs_step_drag(cmbs_t *s, int n_steps, double dragging_steps, cmbs_theory_fn theory_fn, void *user,
                   void *stream) {
    if (!s) return CMBL_ERR_ARG;
    return guarded(&s->last_error, [&] {
        cmamd::sampler_step_drag(s, n_steps, dragging_steps, theory_fn, user, (hipStream_t)stream);
    });
}

int cmbs_history_host(cmbs_t *s, int first, int count, double *out) {
    if (!s || !out || count < 0) return CMBL_ERR_ARG;
    return guarded(&s->last_error, [&] {
        cmamd::sampler_check_pipe(s, true);
        cmamd::sampler_history_host(s, first, count, out);
    });
}

int cmbs_step_theory(cmbs_t *s, int n_steps, cmbs_theory_fn theory_fn, void *user, void *stream) {
    if (!s) return CMBL_ERR_ARG;
    return guarded(&s->last_error,
                   [&] { cmamd::sampler_step_theory(s, n_steps, theory_fn, user, (hipStream_t)stream); });
}

int cmbs_refresh_theory(cmbs_t *s, cmbs_theory_fn theory_fn, void *user, void *stream) {
    if (!s) return CMBL_ERR_ARG;
    return guarded(&s->last_error,
                   [&] { cmamd::sampler_refresh_theory(s, theory_fn, user, (hipStream_t)stream); });
}

int cmbs_collector_enable(cmbs_t *s, int sample_capacity) {
    if (!s) return CMBL_ERR_ARG;
    return guarded(&s->last_error, [&] { cmamd::sampler_collector_enable(s, sample_capacity); });
}

int cmbs_collector_add(cmbs_t *s, const int *steps, int n_steps, int min_sample_update, int check_burn, void *stream) {
    if (!s || (n_steps > 0 && !steps)) return CMBL_ERR_ARG;
    return guarded(&s->last_error, [&] {
        cmamd::sampler_collector_add(s, steps, n_steps, min_sample_update, check_burn, (hipStream_t)stream);
    });
}

int cmbs_collector_state_host(cmbs_t *s, int *start, int *count, int *burn_done, int *thin_fac) {
    if (!s) return CMBL_ERR_ARG;
    return guarded(&s->last_error, [&] { cmamd::sampler_collector_state_host(s, start, count, burn_done, thin_fac); });
}

int cmbs_collector_thin(cmbs_t *s, int limit, void *stream) {
    if (!s) return CMBL_ERR_ARG;
    return guarded(&s->last_error, [&] { cmamd::sampler_collector_thin(s, limit, (hipStream_t)stream); });
}

int cmbs_collector_moments(cmbs_t *s, const double *gmean, double *out, void *stream) {
    if (!s || !out) return CMBL_ERR_ARG;
    return guarded(&s->last_error, [&] { cmamd::sampler_collector_moments(s, gmean, out, (hipStream_t)stream); });
}

int cmbs_collector_limits(cmbs_t *s, const int *params, int n_check, double limfrac, double *out, void *stream) {
    if (!s || (n_check > 0 && (!params || !out))) return CMBL_ERR_ARG;
    return guarded(&s->last_error, [&] {
        cmamd::sampler_collector_limits(s, params, n_check, limfrac, out, (hipStream_t)stream);
    });
}

int cmbs_set_groups(cmbs_t *s, int n_groups) {
    if (!s) return CMBL_ERR_ARG;
    return guarded(&s->last_error, [&] { cmamd::sampler_set_groups(s, n_groups); });
}

int cmbs_set_binned_cache(cmbs_t *s, int on) {
    if (!s) return CMBL_ERR_ARG;
    s->binned_cache = on != 0;
    return CMBL_OK;
}

int cmbs_enable_history(cmbs_t *s, int capacity) {
    if (!s || capacity <= 0) return CMBL_ERR_ARG;
    return guarded(&s->last_error, [&] { cmamd::sampler_enable_history(s, capacity); });
}

int cmbs_history_stats(cmbs_t *s, int first, int last, double *means, double *covs, void *stream) {
    if (!s) return CMBL_ERR_ARG;
    return guarded(&s->last_error,
                   [&] { cmamd::sampler_history_stats(s, first, last, means, covs, (hipStream_t)stream); });
}

int cmbs_history_count(const cmbs_t *s) { return s ? s->hist_count : 0; }

int cmbs_state(cmbs_t *s, double **P, double **cur_like, double **mult, int **num_accept) {
    if (!s) return CMBL_ERR_ARG;
    const auto &R = s->dc.rows;
    const size_t W = s->dc.ld;
    if (P) *P = s->dc.sd + R.P * W;
    if (cur_like) *cur_like = s->dc.sd + R.L * W;
    if (mult) *mult = s->dc.sd + R.M * W;
    if (num_accept) *num_accept = s->dc.si + R.NACC * W;
    return CMBL_OK;
}

int cmbs_get_state_host(cmbs_t *s, double *P, double *cur_like, double *mult, int *num_accept) {
    if (!s) return CMBL_ERR_ARG;
    return guarded(&s->last_error, [&] {
        cmamd::sampler_check_pipe(s, true);
        cmamd::sampler_get_state_host(s, P, cur_like, mult, num_accept);
    });
}

size_t cmbs_state_bytes(const cmbs_t *s) { return s ? cmamd::sampler_state_bytes(s) : 0; }

int cmbs_save_state(cmbs_t *s, void *buf, size_t bytes) {
    if (!s || !buf) return CMBL_ERR_ARG;
    return guarded(&s->last_error, [&] {
        cmamd::sampler_check_pipe(s, true);
        cmamd::sampler_save_state(s, buf, bytes);
    });
}

int cmbs_history_restore(cmbs_t *s, int first, int count, const double *in, const double *terms) {
    if (!s || (count > 0 && !in)) return CMBL_ERR_ARG;
    return guarded(&s->last_error, [&] { cmamd::sampler_history_restore(s, first, count, in, terms); });
}

int cmbs_history_terms_host(cmbs_t *s, int first, int count, double *out) {
    if (!s || (count > 0 && !out)) return CMBL_ERR_ARG;
    return guarded(&s->last_error, [&] {
        cmamd::sampler_check_pipe(s, true);
        cmamd::sampler_history_terms_host(s, first, count, out);
    });
}

int cmbs_load_state(cmbs_t *s, const void *buf, size_t bytes) {
    if (!s || !buf) return CMBL_ERR_ARG;
    return guarded(&s->last_error, [&] { cmamd::sampler_load_state(s, buf, bytes); });
}

}  // extern "C"
