"""Host mirror of CosmoMC's CMB data-likelihood interface for the fast path.

Reference interface (SouthPoleTelescope/CosmoMC):
  * ``TDataLikelihood`` / ``TCMBLikelihood`` -- name, tag, speed, nuisance
    params, ``cl_lmax``, ``GetLogLike(Params, Theory, DataParams)``
    (source/GeneralTypes.f90:105-126, source/Likelihood_Cosmology.f90:148-253)
  * ``CMBLikelihood_Add(LikeList, Ini)`` -- one likelihood per
    ``cmb_dataset[TAG] = file.dataset`` with per-tag overrides
    ``cmb_dataset[TAG,key] = value`` and ``cmb_dataset_speed[TAG]``
    (source/CMB.f90:54-123)
  * ``TLikelihoodList`` with nuisance-parameter index assignment
    (source/GeneralTypes.f90:129-144, 618-669)
  * ``clik_readParams`` / ``clik_lnlike`` (source/cliklike.f90:38-170)

Here every ``LogLike`` is batched over walkers and runs through the HIP
library (cosmomc_amd/lib/libcosmomc_amd.so); theory and nuisance arrays are
torch cuda tensors (device memory, the current HIP stream).
"""
from __future__ import annotations

import ctypes as C
import os
import re

from . import _native as N
from .ini import IniFile

LOGZERO = N.CMBL_LOGZERO
FIELD_INDEX = {"TT": 0, "TE": 1, "EE": 2, "BT": 3, "BE": 4, "BB": 5, "PT": 6, "PE": 7, "PB": 8, "PP": 9}


class DataLikelihood:
    """Base of the fast-path likelihoods (mirrors TDataLikelihood)."""
    LikelihoodType = "CMB"

    def __init__(self):
        self.name = ""
        self.tag = ""
        self.speed = -1                 # TCMBLikelihood_ReadParams (Likelihood_Cosmology.f90:250-251)
        self.nuisance_names: list[str] = []
        self.derived_names: list[str] = []      # the '*' names of the nuisance .paramnames
        self.nuisance_indices: list[int] = []   # 1-based into P, filled by LikelihoodList
        self.dependent_params: set[int] = set()
        self.cl_lmax = [[0] * 4 for _ in range(4)]
        self.version = ""

    def get_tag(self) -> str:
        """TDataLikelihood_GetTag (GeneralTypes.f90:533-543): the tag, else the name."""
        return self.tag or self.name.strip()

    def description(self) -> tuple:
        """(tag, type, name, version): a root.likelihoods line / ChainWriter likelihoods entry."""
        return (self.get_tag(), self.LikelihoodType, self.name, self.version)

    @property
    def n_nuis(self) -> int:
        return len(self.nuisance_names)

    def loglike_batch(self, dl, nuis, out=None):
        raise NotImplementedError


class NativeCMBLikelihood(DataLikelihood):
    """A dataset opened in the HIP library (``cmbl_open``)."""

    def __init__(self, tag: str, dataset: str, overrides: dict | None = None):
        super().__init__()
        text = "".join(f"{k} = {v}\n" for k, v in (overrides or {}).items())
        h = C.c_void_p()
        err = C.create_string_buffer(1024)
        rc = N.lib().cmbl_open(tag.encode(), dataset.encode(), text.encode(), C.byref(h), err, 1024)
        if rc != 0:
            raise N.NativeError(rc, err.value.decode())
        self._h = h
        self.tag = tag
        n_nuis, speed = C.c_int(), C.c_int()
        lm = (C.c_int * 16)()
        name, names = C.c_char_p(), C.c_char_p()
        N.check(N.lib().cmbl_info(h, C.byref(n_nuis), lm, C.byref(speed), C.byref(name), C.byref(names)))
        self.name = name.value.decode()
        self.speed = speed.value
        self.nuisance_names = names.value.decode().split()
        self.cl_lmax = [[lm[i * 4 + j] for j in range(4)] for i in range(4)]
        nd, dnames = C.c_int(), C.c_char_p()
        N.check(N.lib().cmbl_derived_info(h, C.byref(nd), C.byref(dnames)))
        self.derived_names = dnames.value.decode().split()

    @property
    def handle(self):
        return self._h

    def lmax_needed(self) -> int:
        return max(max(r) for r in self.cl_lmax)

    def workspace_bytes(self, W: int) -> int:
        return N.lib().cmbl_workspace_size(self._h, W)

    def loglike_batch(self, dl, nuis, out=None, workspace=None):
        """-lnL for every walker.

        dl   : cuda float64 tensor [W, 10, L] (or [W, nf>=3, L] for plik_lite),
               D_l in muK^2 indexed from l = 0 (field order TT TE EE BT BE BB PT PE PB PP)
        nuis : cuda float64 tensor [W, n_nuis] (DataParams)
        workspace : optional cuda tensor of >= workspace_bytes(W) bytes; default:
               the handle's own
        """
        import torch
        W = dl.shape[0]
        if out is None:
            out = torch.empty(W, dtype=torch.float64, device=dl.device)
        if dl.dtype != torch.float64 or nuis.dtype != torch.float64 or not (dl.is_cuda and nuis.is_cuda):
            raise TypeError("dl and nuis must be float64 cuda tensors")
        if dl.stride(2) != 1 or (nuis.numel() > 0 and nuis.stride(1) != 1):
            raise ValueError("dl rows (l) and nuisance rows must be contiguous")
        ws = workspace.data_ptr() if workspace is not None else None
        nptr, nld = (nuis.data_ptr(), nuis.stride(0)) if nuis.numel() > 0 else (None, 0)
        rc = N.lib().cmbl_loglike_batch(self._h, W, dl.data_ptr(), dl.stride(1), dl.stride(0), nptr, nld,
                                        out.data_ptr(), ws, N.current_stream_ptr(dl.device))
        N.check(rc, self._h)
        return out

    def derived_batch(self, nuis, out=None):
        """derivedParameters(Theory, DataParams) for every walker
        (cmbl_derived_batch; GeneralTypes.f90:504-512, SMICA CMBlikes.f90:1324-1337):
        nuis cuda float64 [W, n_nuis] -> [W, n_derived] on the current stream."""
        import torch
        W, nd = nuis.shape[0], len(self.derived_names)
        if out is None:
            out = torch.empty((W, nd), dtype=torch.float64, device=nuis.device)
        if nd == 0 or W == 0:
            return out
        if nuis.dtype != torch.float64 or not nuis.is_cuda or (nuis.shape[1] > 1 and nuis.stride(1) != 1) or \
                (nd > 1 and out.stride(1) != 1):
            raise TypeError("nuis must be a float64 cuda tensor with contiguous rows")
        rc = N.lib().cmbl_derived_batch(self._h, W, nuis.data_ptr(), nuis.stride(0), out.data_ptr(), out.stride(0),
                                        N.current_stream_ptr(nuis.device))
        N.check(rc, self._h)
        return out

    def status(self, clear: bool = True) -> int:
        """Sticky numerical status bits of the handle (cmbl_status; synchronises):
        CMBL_STATUS_HL_NOCONV = 1 when an HL eigensolve hit its sweep cap since
        the last clear (that walker's -lnL is NaN); CMBL_STATUS_PIPE_WAIT = 2 when
        a sampler's pipelined fast step gave up waiting for its walkers' trial
        calibrations (a safety net; its terms are not to be trusted)."""
        f = C.c_int()
        N.check(N.lib().cmbl_status(self._h, C.byref(f), int(clear)), self._h)
        return f.value

    def loglike_host(self, dl, nuis):
        """Host numpy arrays in/out (PCIe-staged; cmbl_loglike_batch_host)."""
        import numpy as np
        dl = np.ascontiguousarray(dl, dtype=np.float64)
        nuis = np.ascontiguousarray(nuis, dtype=np.float64)
        out = np.empty(dl.shape[0])
        rc = N.lib().cmbl_loglike_batch_host(self._h, dl.shape[0], dl.ctypes.data, dl.shape[2], dl.shape[1] * dl.shape[2],
                                             nuis.ctypes.data, nuis.shape[1], out.ctypes.data)
        N.check(rc, self._h)
        return out

    def close(self):
        if getattr(self, "_h", None):
            N.lib().cmbl_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ClikLikelihood(NativeCMBLikelihood):
    """``clik_data_TAG`` routed to the native kernel (cliklike.f90:129-170).

    The clik library (plc-2.0) is not available; only clik files that are
    plik_lite can be served, from the equivalent native ``.dataset``
    (``clik_native_dataset_TAG`` in the ini).  Results are parity-unpinned
    against real clik.
    """

    def clik_workspace(self, W: int):
        """A device workspace for clik_compute on W rows (cmbl_clik_workspace_size)."""
        import torch
        n = N.lib().cmbl_clik_workspace_size(self._h, W)
        return torch.empty(max(n, 8), dtype=torch.uint8, device="cuda")

    def clik_compute(self, cl_and_pars, clik_lmax, workspace=None):
        """+lnL for rows of the clik vector (device tensor [W, n]); asynchronous."""
        import torch
        W = cl_and_pars.shape[0]
        lm = (C.c_int * 6)(*clik_lmax)
        out = torch.empty(W, dtype=torch.float64, device=cl_and_pars.device)
        ws = workspace.data_ptr() if workspace is not None else None
        rc = N.lib().cmbl_clik_compute_batch(self._h, W, lm, cl_and_pars.data_ptr(), cl_and_pars.stride(0),
                                             out.data_ptr(), ws, N.current_stream_ptr(cl_and_pars.device))
        N.check(rc, self._h)
        return out


def _tag_re(prefix):
    return re.compile(r"^" + re.escape(prefix) + r"\[([^,\]]+)\]$")


def cmb_likelihood_add(like_list: "LikelihoodList", ini: IniFile):
    """CMBLikelihood_Add (source/CMB.f90:54-123) for the natively supported tags."""
    pat = _tag_re("cmb_dataset")
    for key in ini.keys():
        m = pat.match(key)
        if not m:
            continue
        tag = m.group(1)
        fname = ini.relative_filename(key)
        over = {}
        opat = re.compile(r"^cmb_dataset\[" + re.escape(tag) + r",(.+)\]$")
        for k2 in ini.keys():
            mo = opat.match(k2)
            if mo:
                over[mo.group(1)] = ini[k2]
        native_tag = tag if tag in ("PLIK_LITE",) else tag
        like = NativeCMBLikelihood(native_tag, fname, over)
        spd = ini.get(f"cmb_dataset_speed[{tag}]")
        if spd is not None:
            like.speed = int(spd)
        like_list.add(like)
    # clik_data_TAG (cliklike.f90:47-79): natively served when a plik_lite
    # dataset equivalent is given
    for key in ini.keys():
        if not key.startswith("clik_data_"):
            continue
        tag = key[len("clik_data_"):]
        nat = ini.get(f"clik_native_dataset_{tag}")
        if nat is None:
            raise NotImplementedError(f"{key}: the clik library is not available; give "
                                      f"clik_native_dataset_{tag} = <plik_lite .dataset> to use the native kernel")
        like = ClikLikelihood("PLIK_LITE", ini.resolve(nat))
        like.tag = tag
        like.speed = int(ini.get(f"clik_speed_{tag}", "0"))
        pfile = ini.get(f"clik_params_{tag}")
        if pfile:
            like.nuisance_names = read_paramnames(ini.resolve(pfile))
        like_list.add(like)


def read_paramnames(path: str) -> list[str]:
    names = []
    with open(path) as f:
        for line in f:
            t = line.split()
            if t and not t[0].startswith("#"):
                names.append(t[0].rstrip("*"))
    return names


class LikelihoodList:
    """TLikelihoodList: ordered by speed, nuisance indices assigned after the
    theory parameters (AddNuisanceParameters, GeneralTypes.f90:618-669)."""

    def __init__(self):
        self.items: list[DataLikelihood] = []

    def add(self, like: DataLikelihood):
        self.items.append(like)

    def __iter__(self):
        return iter(self.items)

    def __len__(self):
        return len(self.items)

    def add_nuisance_parameters(self, param_names: list[str]) -> list[str]:
        """Sort by speed (stable, CompareLikes :602-615) and give every likelihood
        contiguous 1-based nuisance indices; returns the extended name list."""
        self.items.sort(key=lambda l: l.speed)
        names = list(param_names)
        self.derived_list = []
        self.first_fast_param = 0
        for like in self.items:
            like.new_param_block_start = len(names) + 1          # :638
            idx = []
            for nm in like.nuisance_names:
                if nm in names:
                    idx.append(names.index(nm) + 1)
                else:
                    names.append(nm)                             # ParamNames_Add: new names only
                    idx.append(len(names))
            like.new_params = len(names) - like.new_param_block_start + 1   # :641
            like.nuisance_indices = idx
            # derived names follow every MCMC name (ParamNames_Add orders non-derived
            # first); derived_indices (:658-664) are 1-based into the derived list
            like.derived_indices = []
            for nm in like.derived_names:
                if nm not in self.derived_list:
                    self.derived_list.append(nm)
                like.derived_indices.append(self.derived_list.index(nm) + 1)
            like.dependent_params = set(idx)
            if self.first_fast_param == 0 and like.speed >= 0 and like.new_params > 0 and idx:   # :650-651
                self.first_fast_param = like.new_param_block_start
        return names
