"""ORACLE TEST INFRASTRUCTURE -- ctypes view of oracle/liboracle.so.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, as the checker / CPU baseline.  Nothing in cosmomc_amd/ does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

_dp = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_ip = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_lp = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")


class Rng(C.Structure):
    _fields_ = [("u", C.c_double * 97), ("c", C.c_double), ("cd", C.c_double), ("cm", C.c_double),
                ("i97", C.c_int), ("j97", C.c_int), ("iset", C.c_int), ("gset", C.c_double)]


class DragState(C.Structure):
    _fields_ = [("num_drag", C.c_int), ("mult", C.c_double), ("dragging_steps", C.c_double),
                ("oversample_fast", C.c_int)]


class Target(C.Structure):
    _fields_ = [("num_params", C.c_int), ("pmin", C.c_void_p), ("pmax", C.c_void_p),
                ("prior_mean", C.c_void_p), ("prior_std", C.c_void_p), ("temperature", C.c_double),
                ("test_like", C.c_int), ("n_used", C.c_int), ("params_used", C.c_void_p),
                ("test_covinv", C.c_void_p), ("center", C.c_void_p), ("plik", C.c_void_p),
                ("plik_nuis_index", C.c_int), ("plik_dl", C.c_void_p), ("plik_ld_field", C.c_long),
                ("plik_scale_index", C.c_int), ("include_fixed_parameter_priors", C.c_int),
                ("varying", C.c_void_p), ("n_lincomb", C.c_int), ("lincomb_weights", C.c_void_p),
                ("lincomb_mean", C.c_void_p), ("lincomb_std", C.c_void_p),
                ("extra_like", C.c_void_p), ("extra_user", C.c_void_p)]


# Target.extra_like: double (*)(void *user, const double *P)
EXTRA_LIKE_FN = C.CFUNCTYPE(C.c_double, C.c_void_p, C.POINTER(C.c_double))


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            subprocess.run(["make", "-C", HERE, "oracle"], check=True, stdout=subprocess.DEVNULL)
        L = C.CDLL(path)
        L.orc_rmarin.argtypes = [C.POINTER(Rng), C.c_int, C.c_int]
        L.orc_ranmar.argtypes = [C.POINTER(Rng)]
        L.orc_ranmar.restype = C.c_double
        L.orc_gaussian1.argtypes = [C.POINTER(Rng)]
        L.orc_gaussian1.restype = C.c_double
        L.orc_randexp1.argtypes = [C.POINTER(Rng)]
        L.orc_randexp1.restype = C.c_float
        L.orc_rand_indices.argtypes = [C.POINTER(Rng), _ip, C.c_int, C.c_int]
        L.orc_rand_rotation.argtypes = [C.POINTER(Rng), _dp, C.c_int]
        L.orc_matrix_inverse.argtypes = [_dp, C.c_int]
        L.orc_matrix_inverse.restype = C.c_int
        L.orc_quadform.argtypes = [_dp, _dp, C.c_int]
        L.orc_quadform.restype = C.c_double
        L.orc_plik_create.argtypes = [C.c_int, C.c_int, _dp, _lp, _lp, C.c_int, _ip, C.c_int, C.c_int,
                                      C.c_int, _dp, _dp, C.c_int]
        L.orc_plik_create.restype = C.c_void_p
        L.orc_plik_nused.argtypes = [C.c_void_p]
        L.orc_plik_loglike.argtypes = [C.c_void_p, C.c_void_p, C.c_long, C.c_double]
        L.orc_plik_loglike.restype = C.c_double
        L.orc_plik_free.argtypes = [C.c_void_p]
        L.orc_proposer_create.argtypes = [C.c_int, _ip, _ip, C.c_int, C.c_int, C.c_double, C.c_int, _ip]
        L.orc_proposer_create.restype = C.c_void_p
        L.orc_proposer_set_covariance.argtypes = [C.c_void_p, _dp]
        for fn in ("orc_proposer_get_proposal", "orc_proposer_get_proposal_slow", "orc_proposer_get_proposal_fast"):
            getattr(L, fn).argtypes = [C.c_void_p, C.POINTER(Rng), _dp]
        L.orc_proposer_get_proposal_fast_delta.argtypes = [C.c_void_p, C.POINTER(Rng), _dp, C.c_int]
        L.orc_proposer_free.argtypes = [C.c_void_p]
        L.orc_target_loglike.argtypes = [C.POINTER(Target), _dp]
        L.orc_target_loglike.restype = C.c_double
        L.orc_metropolis_accept.argtypes = [C.POINTER(Rng), C.c_double, C.c_double]
        L.orc_metropolis_accept.restype = C.c_int
        L.orc_mh_step.argtypes = [C.c_void_p, C.POINTER(Rng), C.POINTER(Target), _dp, C.POINTER(C.c_double),
                                  C.c_int, C.POINTER(C.c_double)]
        L.orc_mh_step.restype = C.c_int
        L.orc_drag_step.argtypes = [C.c_void_p, C.POINTER(Rng), C.POINTER(Target), C.POINTER(DragState), _dp,
                                    C.POINTER(C.c_double)]
        L.orc_drag_step.restype = C.c_int
        L.orc_gelman_rubin.argtypes = [_dp, _dp, C.c_int]
        L.orc_gelman_rubin.restype = C.c_double
        _LIB = L
    return _LIB


class Ranmar:
    """RANMAR stream as RandUtils.f90 (one chain's generator)."""

    def __init__(self, ij: int, kl: int = 9373):
        self.s = Rng()
        lib().orc_rmarin(C.byref(self.s), ij, kl)

    def ranmar(self, n=None):
        if n is None:
            return lib().orc_ranmar(C.byref(self.s))
        return np.array([lib().orc_ranmar(C.byref(self.s)) for _ in range(n)])

    def gaussian1(self):
        return lib().orc_gaussian1(C.byref(self.s))

    def randexp1(self):
        return lib().orc_randexp1(C.byref(self.s))

    def rand_indices(self, nmax, n):
        out = np.zeros(n, dtype=np.int32)
        lib().orc_rand_indices(C.byref(self.s), out, nmax, n)
        return out

    def rand_rotation(self, n):
        R = np.zeros(n * n)
        lib().orc_rand_rotation(C.byref(self.s), R, n)
        return R.reshape(n, n)


class PlikLite:
    """Oracle TPlikLiteLikelihood built from cosmomc_amd.synthetic.PlikLiteData."""
    USE_BITS = {"TT": 1, "TE": 2, "EE": 4}

    def __init__(self, data, use_cl="TT TE EE", bins_for_L_range=None, plmin=30):
        mask = 0
        for tok in use_cl.split():
            mask |= self.USE_BITS[tok]
        rmin, rmax = (-1, -1) if bins_for_L_range is None else bins_for_L_range
        nbincl = np.array([215, 199, 199], dtype=np.int32)
        self._keep = (np.ascontiguousarray(data.weights_file, dtype=np.float64),
                      np.ascontiguousarray(data.blmin, dtype=np.int64),
                      np.ascontiguousarray(data.blmax, dtype=np.int64),
                      np.ascontiguousarray(data.X, dtype=np.float64),
                      np.ascontiguousarray(data.cov, dtype=np.float64))
        w, lo, hi, X, cov = self._keep
        self.h = lib().orc_plik_create(plmin, w.size, w, lo, hi, lo.size, nbincl, mask, rmin, rmax, X, cov, X.size)
        if not self.h:
            raise RuntimeError("oracle plik_lite: covariance not positive definite")
        self.nused = lib().orc_plik_nused(self.h)

    def loglike(self, dl: np.ndarray, cal: float) -> float:
        """dl: [n_fields>=3, ld] float64 for one walker."""
        dl = np.ascontiguousarray(dl, dtype=np.float64)
        return lib().orc_plik_loglike(self.h, dl.ctypes.data, dl.shape[-1], float(cal))

    def loglike_batch(self, dl: np.ndarray, cal: np.ndarray) -> np.ndarray:
        return np.array([self.loglike(dl[i], cal[i]) for i in range(dl.shape[0])])

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_plik_free(self.h)
            self.h = None


def pool_chain_statistics(samples):
    """TMpiChainCollector_UpdateCovAndCheckConverge pooling (SampleCollector.f90:233-286)
    restated with explicit loops: samples [M chains][Count][n]; each chain uses
    Items Count/2 .. Count (1-based, inclusive).  Returns the count-weighted
    pooled mean, MPICovMat (count-weighted mean of the chain covariances, the
    learnt proposal), cov (plain mean of covariances) and meanscov (weighted
    covariance of the chain means times M/(M-1))."""
    M = len(samples)
    n = samples[0].shape[1]
    counts, means, covs = [], [], []
    for x in samples:
        cnt = x.shape[0]
        lo = cnt // 2                       # 1-based Count/2 -> 0-based lo-1
        rows = x[lo - 1:cnt]
        c0 = cnt - cnt // 2 + 1
        m = np.zeros(n)
        for r in rows:
            m += r
        m /= c0
        C = np.zeros((n, n))
        for r in rows:
            d = r - m
            C += np.outer(d, d)
        counts.append(float(c0)); means.append(m); covs.append(C / c0)
    w = np.array(counts)
    norm = w.sum()
    mean = sum(w[c] * means[c] for c in range(M)) / norm
    mpicov = np.zeros((n, n)); cov = np.zeros((n, n)); meanscov = np.zeros((n, n))
    for i in range(n):
        for j in range(i, n):
            mpicov[i, j] = sum(w[c] * covs[c][i, j] for c in range(M)) / norm
            cov[i, j] = sum(covs[c][i, j] for c in range(M)) / M
            meanscov[i, j] = sum(w[c] * (means[c][i] - mean[i]) * (means[c][j] - mean[j]) for c in range(M)) / norm
            mpicov[j, i], cov[j, i], meanscov[j, i] = mpicov[i, j], cov[i, j], meanscov[i, j]
    meanscov = meanscov * M / (M - 1)
    return {"counts": w, "mean": mean, "propose_cov": mpicov, "cov": cov, "meanscov": meanscov}


def gelman_rubin(cov, meanscov):
    """max eigenvalue of GelmanRubinEvalues (samples.f90:41-67); 1e6 if not invertible."""
    n = cov.shape[0]
    return lib().orc_gelman_rubin(np.ascontiguousarray(cov), np.ascontiguousarray(meanscov), n)


def confid_val(values, limfrac, ix1=None, ix2=None):
    """TSampleList%ConfidVal (samples.f90:70-110) of one column: sort items
    ix1..ix2 (1-based, inclusive), interpolate the order statistics at
    pos = (samps-1)*limfrac + 1 and (samps-1)*(1-limfrac) + 1."""
    v = np.asarray(values, dtype=np.float64)
    b0 = 1 if ix1 is None else ix1
    t0 = v.size if ix2 is None else ix2
    x = np.sort(v[b0 - 1:t0])
    samps = t0 - b0 + 1
    out = []
    for frac in (limfrac, 1.0 - limfrac):
        pos = (samps - 1) * frac + 1
        b = max(int(pos), 1)
        val = x[b - 1]
        if b < samps and pos > b:
            d = pos - b
            val = val * (1 - d) + d * x[b]
        out.append(val)
    return out[0], out[1]


def collector_samples(rows, steps, min_update, check_burn=True, thin=1, state=None):
    """One chain's TMpiChainCollector Samples list (SampleCollector.f90:324-397)
    restated item by item: rows[t] = (P_used..., like) of history step t;
    AddNewPoint at each step in `steps` (logZero points skipped, MCMC.f90:146):
    sample_num++, keep every thin-th, Add, burn-in test once Count > 51
    (every parameter changed > 51 times between consecutive items), then
    DeleteRange(1, Count - min_update).  state (dict, updated in place):
    items (history steps), sample_num, burn, changes."""
    st = state if state is not None else {"items": [], "sample_num": 0, "burn": False, "changes": None}
    n = rows.shape[1] - 1
    for t in steps:
        if rows[t, n] == 1e30:
            continue
        st["sample_num"] += 1
        if st["sample_num"] % thin != 0:
            continue
        st["items"].append(t)
        cnt = len(st["items"])
        if st["burn"] or not check_burn or cnt <= 51:
            continue
        if st["changes"] is None:
            st["changes"] = np.zeros(n, dtype=int)
        a, b = rows[st["items"][-1], :n], rows[st["items"][-2], :n]
        st["changes"] += (a != b)
        if np.all(st["changes"] > 51):
            st["burn"] = True
            if cnt > min_update:
                del st["items"][:cnt - min_update]
            st["changes"] = None
    return st
