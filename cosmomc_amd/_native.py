"""ctypes binding of libcosmomc_amd.so (include/cosmomc_amd.h).

The HIP library is the only compute path: there is no CPU fallback.  Loading
fails loudly if the library is missing; compute calls fail loudly without a
GPU.
"""
from __future__ import annotations

import ctypes as C
import os
import re
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
# COSMOMC_AMD_LIB selects an instrumented build of the same sources (tools/)
LIB_PATH = os.environ.get("COSMOMC_AMD_LIB") or os.path.join(PKG, "lib", "libcosmomc_amd.so")
HEADER = os.path.join(ROOT, "include", "cosmomc_amd.h")

CMBL_LOGZERO = 1e30
N_FIELDS = 10

ERRORS = {0: "OK", -1: "bad argument", -2: "I/O error", -3: "format error", -4: "numerical error",
          -5: "HIP error", -6: "unsupported"}


class NativeError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"[{ERRORS.get(code, code)}] {msg}")
        self.code = code


class CmbsConfig(C.Structure):
    _fields_ = [("n_walkers", C.c_int), ("num_params", C.c_int), ("n_used", C.c_int),
                ("params_used", C.POINTER(C.c_int)), ("n_blocks", C.c_int), ("block_n", C.POINTER(C.c_int)),
                ("block_params", C.POINTER(C.c_int)), ("slow_block_max", C.c_int), ("oversample_fast", C.c_int),
                ("propose_scale", C.c_double), ("temperature", C.c_double),
                ("pmin", C.POINTER(C.c_double)), ("pmax", C.POINTER(C.c_double)),
                ("prior_mean", C.POINTER(C.c_double)), ("prior_std", C.POINTER(C.c_double)),
                ("seed_ij", C.c_int), ("seed_kl", C.c_int), ("first_walker", C.c_int),
                ("include_fixed_parameter_priors", C.c_int), ("n_lincomb", C.c_int),
                ("lincomb_weights", C.POINTER(C.c_double)), ("lincomb_mean", C.POINTER(C.c_double)),
                ("lincomb_std", C.POINTER(C.c_double))]


_lib = None

# cmbs_theory_fn: int (*)(void *user, int W, const double *P_end, long long ld, void *stream)
THEORY_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_longlong, C.c_void_p)


class DeviceRows:
    """__cuda_array_interface__ view of device rows [n][ld] (walker-minor), for
    torch.as_tensor without a copy."""

    def __init__(self, ptr, n, W, ld):
        self.__cuda_array_interface__ = {"shape": (n, W), "typestr": "<f8", "data": (ptr, False),
                                         "strides": (ld * 8, 8), "version": 2}


def build(force: bool = False) -> str:
    """Compile the HIP library in-tree (hipcc --offload-arch=gfx950)."""
    if force or not os.path.exists(LIB_PATH):
        jobs = str(min(16, os.cpu_count() or 4))
        subprocess.run(["make", "-C", os.path.join(PKG, "csrc"), "-j" + jobs], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"cosmomc_amd native library missing ({LIB_PATH}); run "
                              "`make -C cosmomc_amd/csrc` or __graft_entry__.build()")
        L = C.CDLL(LIB_PATH)
        vp, i, ll, d, sz = C.c_void_p, C.c_int, C.c_longlong, C.c_double, C.c_size_t
        L.cmbl_open.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.POINTER(vp), C.c_char_p, sz]
        L.cmbl_close.argtypes = [vp]
        L.cmbl_last_error.argtypes = [vp]
        L.cmbl_last_error.restype = C.c_char_p
        L.cmbl_info.argtypes = [vp, C.POINTER(i), C.POINTER(i), C.POINTER(i), C.POINTER(C.c_char_p),
                                C.POINTER(C.c_char_p)]
        L.cmbl_derived_info.argtypes = [vp, C.POINTER(i), C.POINTER(C.c_char_p)]
        L.cmbl_derived_batch.argtypes = [vp, i, vp, ll, vp, ll, vp]
        L.cmbl_workspace_size.argtypes = [vp, i]
        L.cmbl_workspace_size.restype = sz
        L.cmbl_loglike_batch.argtypes = [vp, i, vp, ll, ll, vp, ll, vp, vp, vp]
        L.cmbl_loglike_batch_host.argtypes = [vp, i, vp, ll, ll, vp, ll, vp]
        L.cmbl_clik_compute_batch.argtypes = [vp, i, vp, vp, ll, vp, vp, vp]
        L.cmbl_clik_workspace_size.argtypes = [vp, i]
        L.cmbl_clik_workspace_size.restype = sz
        L.cmbl_status.argtypes = [vp, C.POINTER(i), i]
        L.cmbs_walker_seed.argtypes = [i, i, i, C.POINTER(i), C.POINTER(i)]
        L.cmbs_create.argtypes = [C.POINTER(CmbsConfig), C.POINTER(vp), C.c_char_p, sz]
        L.cmbs_destroy.argtypes = [vp]
        L.cmbs_last_error.argtypes = [vp]
        L.cmbs_last_error.restype = C.c_char_p
        L.cmbs_set_covariance.argtypes = [vp, vp]
        L.cmbs_set_test_gaussian.argtypes = [vp, vp, vp]
        L.cmbs_add_likelihood.argtypes = [vp, vp, vp, vp, ll, ll]
        L.cmbs_set_start.argtypes = [vp, vp, vp]
        L.cmbs_step.argtypes = [vp, i, i, vp]
        L.cmbs_set_groups.argtypes = [vp, i]
        L.cmbs_set_binned_cache.argtypes = [vp, i]
        L.cmbs_history_host.argtypes = [vp, i, i, vp]
        L.cmbs_set_trial_theory.argtypes = [vp, i, vp, ll, ll]
        L.cmbs_step_drag.argtypes = [vp, i, d, THEORY_FN, vp, vp]
        L.cmbs_step_theory.argtypes = [vp, i, THEORY_FN, vp, vp]
        L.cmbs_refresh_theory.argtypes = [vp, THEORY_FN, vp, vp]
        L.cmbs_collector_enable.argtypes = [vp, i]
        L.cmbs_collector_add.argtypes = [vp, vp, i, i, i, vp]
        L.cmbs_collector_state_host.argtypes = [vp, vp, vp, vp, vp]
        L.cmbs_collector_thin.argtypes = [vp, i, vp]
        L.cmbs_collector_moments.argtypes = [vp, vp, vp, vp]
        L.cmbs_collector_limits.argtypes = [vp, vp, i, d, vp, vp]
        L.cmbs_chain_moments.argtypes = [vp, i, i, vp, vp, vp]
        L.cmbs_enable_history.argtypes = [vp, i]
        L.cmbs_history_stats.argtypes = [vp, i, i, vp, vp, vp]
        L.cmbs_history_count.argtypes = [vp]
        L.cmbs_state.argtypes = [vp, C.POINTER(vp), C.POINTER(vp), C.POINTER(vp), C.POINTER(vp)]
        L.cmbs_get_state_host.argtypes = [vp, vp, vp, vp, vp]
        L.cmbs_state_bytes.argtypes = [vp]
        L.cmbs_state_bytes.restype = sz
        L.cmbs_save_state.argtypes = [vp, vp, sz]
        L.cmbs_load_state.argtypes = [vp, vp, sz]
        L.cmbs_history_restore.argtypes = [vp, i, i, vp, vp]
        L.cmbs_history_terms_host.argtypes = [vp, i, i, vp]
        L.cmbl_profile_enable.argtypes = [i]
        L.cmbl_profile_reset.argtypes = []
        L.cmbl_profile_read.argtypes = [C.c_char_p, C.POINTER(d), C.POINTER(ll)]
        _lib = L
    return _lib


def exported_symbols_from_header() -> list[str]:
    """Function names declared in include/cosmomc_amd.h."""
    with open(HEADER) as f:
        txt = f.read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(cmb[ls]_[a-z_0-9]+)\s*\(", txt)))


def check(rc: int, handle=None, kind: str = "cmbl"):
    if rc != 0:
        msg = ""
        if handle is not None:
            fn = lib().cmbl_last_error if kind == "cmbl" else lib().cmbs_last_error
            msg = (fn(handle) or b"").decode()
        raise NativeError(rc, msg)


def current_stream_ptr(device=None) -> int:
    import torch
    if device is None:   # the raw handle without a Stream object: a few us less per step call
        try:
            return torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice())
        except AttributeError:
            pass
    return torch.cuda.current_stream(device).cuda_stream


def require_gpu():
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError("cosmomc_amd compute needs an MI355X (HIP) device; none visible")


def profile_enable(on: bool = True):
    lib().cmbl_profile_enable(int(on))


def profile_reset():
    lib().cmbl_profile_reset()


def profile_read(kernel: str):
    """(total_ms, launches) of a library kernel since the last reset."""
    t, n = C.c_double(), C.c_longlong()
    lib().cmbl_profile_read(kernel.encode(), C.byref(t), C.byref(n))
    return t.value, n.value
