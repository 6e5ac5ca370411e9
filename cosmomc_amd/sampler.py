"""Batched CosmoMC Metropolis sampler on the GPU (host wrapper of ``cmbs_*``).

Mirrors TChainSampler / TMetropolisSampler (reference source/MCMC.f90:34-335)
with a BlockedProposer (source/propose.f90) per walker: W independent chains
that each follow the reference's per-chain random-number call order, so
walker w seeded (ij_w, kl_w) = ``walker_seed(ij, kl, w)`` reproduces the
reference chain started with those seeds.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _native as N


def walker_seed(seed_ij: int, seed_kl: int, walker: int) -> tuple[int, int]:
    ij, kl = C.c_int(), C.c_int()
    N.lib().cmbs_walker_seed(seed_ij, seed_kl, walker, C.byref(ij), C.byref(kl))
    return ij.value, kl.value


def _ia(x):
    a = np.ascontiguousarray(x, dtype=np.int32)
    return a, a.ctypes.data_as(C.POINTER(C.c_int))


def _da(x):
    a = np.ascontiguousarray(x, dtype=np.float64)
    return a, a.ctypes.data_as(C.POINTER(C.c_double))


class BatchedMCMC:
    def __init__(self, n_walkers: int, num_params: int, params_used, blocks, slow_block_max: int,
                 pmin, pmax, prior_mean=None, prior_std=None, oversample_fast: int = 1,
                 propose_scale: float = 2.4, temperature: float = 1.0, seed_ij: int = 1802,
                 seed_kl: int = 9373, first_walker: int = 0, include_fixed_parameter_priors: bool = False,
                 linear_combinations=None):
        """linear_combinations: [(weights[num_params], mean, std), ...] priors on
        dot(weights, P) (BaseParams%LinearCombinations, BaseParameters.f90:184-201)."""
        self.W, self.np = n_walkers, num_params
        self.params_used = list(params_used)
        self.pmin = np.array(pmin, dtype=np.float64)
        self.pmax = np.array(pmax, dtype=np.float64)
        self._keep = []
        cfg = N.CmbsConfig()
        cfg.n_walkers, cfg.num_params, cfg.n_used = n_walkers, num_params, len(self.params_used)
        a, cfg.params_used = _ia(self.params_used); self._keep.append(a)
        cfg.n_blocks = len(blocks)
        a, cfg.block_n = _ia([len(b) for b in blocks]); self._keep.append(a)
        a, cfg.block_params = _ia([x for b in blocks for x in b] or [0]); self._keep.append(a)
        cfg.slow_block_max, cfg.oversample_fast = slow_block_max, oversample_fast
        cfg.propose_scale, cfg.temperature = propose_scale, temperature
        a, cfg.pmin = _da(pmin); self._keep.append(a)
        a, cfg.pmax = _da(pmax); self._keep.append(a)
        pm = np.zeros(num_params) if prior_mean is None else prior_mean
        ps = np.zeros(num_params) if prior_std is None else prior_std
        a, cfg.prior_mean = _da(pm); self._keep.append(a)
        a, cfg.prior_std = _da(ps); self._keep.append(a)
        cfg.seed_ij, cfg.seed_kl, cfg.first_walker = seed_ij, seed_kl, first_walker
        cfg.include_fixed_parameter_priors = int(bool(include_fixed_parameter_priors))
        lin = list(linear_combinations or [])
        cfg.n_lincomb = len(lin)
        if lin:
            a, cfg.lincomb_weights = _da(np.array([np.asarray(l[0], dtype=np.float64) for l in lin]))
            self._keep.append(a)
            a, cfg.lincomb_mean = _da([float(l[1]) for l in lin]); self._keep.append(a)
            a, cfg.lincomb_std = _da([float(l[2]) for l in lin]); self._keep.append(a)
        h = C.c_void_p()
        err = C.create_string_buffer(1024)
        rc = N.lib().cmbs_create(C.byref(cfg), C.byref(h), err, 1024)
        if rc:
            raise N.NativeError(rc, err.value.decode())
        self._h = h
        self._likes = []

    def _check(self, rc):
        N.check(rc, self._h, "cmbs")

    def set_covariance(self, cov):
        c = np.ascontiguousarray(cov, dtype=np.float64)
        self._check(N.lib().cmbs_set_covariance(self._h, c.ctypes.data))

    def set_test_gaussian(self, cov, center):
        c = np.ascontiguousarray(cov, dtype=np.float64)
        m = np.ascontiguousarray(center, dtype=np.float64)
        self._check(N.lib().cmbs_set_test_gaussian(self._h, c.ctypes.data, m.ctypes.data))

    def add_likelihood(self, like, dl):
        """like: NativeCMBLikelihood with nuisance_indices set (1-based indices
        into P, any order, GeneralTypes.f90:642-646); dl: cuda tensor [W, nf, L]."""
        idx = np.ascontiguousarray(list(like.nuisance_indices) or [0], dtype=np.int32)
        self._likes.append((like, dl))
        self._check(N.lib().cmbs_add_likelihood(self._h, like.handle, idx.ctypes.data, dl.data_ptr(), dl.stride(1),
                                                dl.stride(0)))

    def set_start(self, P0, stream=None):
        p = np.ascontiguousarray(P0, dtype=np.float64).reshape(self.W, self.np)
        self._check(N.lib().cmbs_set_start(self._h, p.ctypes.data, stream))

    def set_binned_cache(self, on: bool = True):
        """Bin each walker's theory once per fast-step call and reuse the raw
        sums at every step (cmbs_set_binned_cache; SURVEY 8(d)'s labelled
        variant: same results, less work per step -- never the headline)."""
        self._check(N.lib().cmbs_set_binned_cache(self._h, int(bool(on))))

    def set_groups(self, n_groups: int):
        """Step the walkers as ``n_groups`` slices on concurrent internal
        streams (cmbs_set_groups; execution tuning, results unchanged)."""
        self._check(N.lib().cmbs_set_groups(self._h, int(n_groups)))

    def step(self, n_steps: int = 1, fast_only: bool = False, stream=None):
        if stream is None:
            stream = N.current_stream_ptr()
        self._check(N.lib().cmbs_step(self._h, n_steps, int(fast_only), stream))

    def set_trial_theory(self, like_index: int, dl_end):
        """Trial-point theory buffer of likelihood ``like_index`` (cuda float64
        tensor shaped like the theory given to add_likelihood), filled by the
        theory function of step_drag / step_theory."""
        self._drag_keep = getattr(self, "_drag_keep", {})
        self._drag_keep[like_index] = dl_end
        self._check(N.lib().cmbs_set_trial_theory(self._h, like_index, dl_end.data_ptr(), dl_end.stride(1),
                                                  dl_end.stride(0)))

    set_drag_theory = set_trial_theory

    def _theory_cb(self, theory_fn):
        import torch
        if theory_fn is None:
            return N.THEORY_FN()

        def _cb(user, W, ptr, ld, strm):
            try:
                theory_fn(torch.as_tensor(N.DeviceRows(ptr, self.np, W, ld), device="cuda"))
                return 0
            except Exception:                        # reported as a failed theory call
                import traceback
                traceback.print_exc()
                return 1
        return N.THEORY_FN(_cb)

    def step_theory(self, n_steps: int = 1, theory_fn=None, stream=None):
        """n_steps full GetNewSample steps (slow and fast proposals) with the
        theory at every trial point from theory_fn(P_trial [num_params, W])."""
        if stream is None:
            stream = N.current_stream_ptr()
        cb = self._theory_cb(theory_fn)
        self._check(N.lib().cmbs_step_theory(self._h, n_steps, cb, None, stream))

    def step_drag(self, n_steps: int = 1, dragging_steps: float = 3.0, theory_fn=None, stream=None):
        """n_steps TFastDraggingSampler_GetNewSample calls (MCMC.f90:338-452).

        theory_fn(P_end) -> None fills every end-theory buffer (set_drag_theory)
        for the proposed points P_end, a cuda tensor view [num_params, W]."""
        if stream is None:
            stream = N.current_stream_ptr()
        cb = self._theory_cb(theory_fn)
        self._check(N.lib().cmbs_step_drag(self._h, n_steps, dragging_steps, cb, None, stream))

    def refresh_theory(self, theory_fn, stream=None):
        """After load_state of a run that moved slow parameters: theory_fn(P
        [num_params, W]) fills the trial-theory buffers at the current points,
        which become the walkers' theory (cmbs_refresh_theory)."""
        if stream is None:
            stream = N.current_stream_ptr()
        cb = self._theory_cb(theory_fn)
        self._check(N.lib().cmbs_refresh_theory(self._h, cb, None, stream))

    def enable_history(self, capacity: int):
        self._check(N.lib().cmbs_enable_history(self._h, capacity))
        self._hist_cap = capacity

    def history_count(self) -> int:
        return N.lib().cmbs_history_count(self._h)

    def history_host(self, first: int, count: int):
        """History rows [first, first+count) on the host: [count, n_used + 1, W]
        (used parameters, then CurLike)."""
        out = np.empty((count, len(self.params_used) + 1, self.W))
        self._check(N.lib().cmbs_history_host(self._h, first, count, out.ctypes.data))
        return out

    def history_terms(self, first: int, count: int):
        """Each likelihood's -lnL at history rows [first, first+count) on the
        host: [count, n_likelihoods, W] (add_likelihood order)."""
        out = np.empty((count, len(self._likes), self.W))
        if self._likes:
            self._check(N.lib().cmbs_history_terms_host(self._h, first, count, out.ctypes.data))
        return out

    def history_stats(self, first: int, last: int):
        """Per-walker means [W, n_used] and covariances [W, n_used, n_used] (cuda tensors)."""
        import torch
        n = len(self.params_used)
        means = torch.empty((self.W, n), dtype=torch.float64, device="cuda")
        covs = torch.empty((self.W, n, n), dtype=torch.float64, device="cuda")
        self._check(N.lib().cmbs_history_stats(self._h, first, last, means.data_ptr(), covs.data_ptr(),
                                               N.current_stream_ptr()))
        return means, covs

    def chain_moments(self, first: int, last: int, gmean=None):
        """This GPU's partial sums for the convergence exchange (cmbs_chain_moments)."""
        import torch
        n = len(self.params_used)
        out = torch.empty(2 + n + 2 * n * n if gmean is None else n * n, dtype=torch.float64, device="cuda")
        g = None
        if gmean is not None:
            g = torch.as_tensor(gmean, dtype=torch.float64, device="cuda").contiguous()
        self._check(N.lib().cmbs_chain_moments(self._h, first, last, None if g is None else g.data_ptr(),
                                               out.data_ptr(), N.current_stream_ptr()))
        return out

    # ---- sample collector (cmbs_collector_*; cosmomc_amd.converge.ChainCollector drives it)
    def collector_enable(self, sample_capacity: int):
        self._check(N.lib().cmbs_collector_enable(self._h, int(sample_capacity)))

    def collector_add(self, steps, min_sample_update: int, check_burn: bool = True):
        st = np.ascontiguousarray(steps, dtype=np.int32)
        if st.size:
            self._check(N.lib().cmbs_collector_add(self._h, st.ctypes.data, st.size, int(min_sample_update),
                                                   int(check_burn), N.current_stream_ptr()))

    def collector_state(self):
        """Per-walker (start, count, burn_done, thin_fac) host int arrays."""
        a = [np.empty(self.W, dtype=np.int32) for _ in range(4)]
        self._check(N.lib().cmbs_collector_state_host(self._h, *[x.ctypes.data for x in a]))
        return tuple(a)

    def collector_thin(self, limit: int):
        self._check(N.lib().cmbs_collector_thin(self._h, int(limit), N.current_stream_ptr()))

    def collector_moments(self, gmean=None):
        import torch
        n = len(self.params_used)
        out = torch.empty(2 + n + 2 * n * n if gmean is None else n * n, dtype=torch.float64, device="cuda")
        g = None if gmean is None else torch.as_tensor(gmean, dtype=torch.float64, device="cuda").contiguous()
        self._check(N.lib().cmbs_collector_moments(self._h, None if g is None else g.data_ptr(), out.data_ptr(),
                                                   N.current_stream_ptr()))
        return out

    def collector_limits(self, params, limfrac: float):
        """[W, len(params), 2] device tensor of (lower, upper) ConfidVal limits."""
        import torch
        p = np.ascontiguousarray(params, dtype=np.int32)
        out = torch.empty((self.W, p.size, 2), dtype=torch.float64, device="cuda")
        self._check(N.lib().cmbs_collector_limits(self._h, p.ctypes.data, p.size, float(limfrac), out.data_ptr(),
                                                  N.current_stream_ptr()))
        return out

    device = "cuda"

    def state(self):
        P = np.empty((self.W, self.np))
        like = np.empty(self.W)
        mult = np.empty(self.W)
        nacc = np.empty(self.W, dtype=np.int32)
        self._check(N.lib().cmbs_get_state_host(self._h, P.ctypes.data, like.ctypes.data, mult.ctypes.data,
                                                nacc.ctypes.data))
        return P, like, mult, nacc

    def save_state(self) -> bytes:
        """Every walker's complete chain state (cmbs_save_state): point,
        CurLike, multiplicity, accept count, RANMAR and proposer state."""
        n = N.lib().cmbs_state_bytes(self._h)
        buf = C.create_string_buffer(n)
        self._check(N.lib().cmbs_save_state(self._h, buf, n))
        return buf.raw

    def load_state(self, image: bytes):
        """Resume from save_state's image (set_covariance first); replaces set_start."""
        buf = C.create_string_buffer(bytes(image), len(image))
        self._check(N.lib().cmbs_load_state(self._h, buf, len(image)))

    def history_restore(self, first: int, rows, terms=None):
        """Put history rows [first, first + len(rows)) back (layouts of
        history_host / history_terms)."""
        r = np.ascontiguousarray(rows, dtype=np.float64)
        t = None if terms is None else np.ascontiguousarray(terms, dtype=np.float64)
        self._check(N.lib().cmbs_history_restore(self._h, first, r.shape[0], r.ctypes.data,
                                                 None if t is None else t.ctypes.data))

    def close(self):
        if getattr(self, "_h", None):
            N.lib().cmbs_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
