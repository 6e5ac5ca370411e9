"""ORACLE TEST INFRASTRUCTURE -- never shipped, never on the product path.

numpy restatement of the reference's CMBlikes bandpower likelihood
(source/CMBlikes.f90), the BICEP/Keck/Planck foreground model
(source/CMB_BK_Planck.f90) and the SMICA TT foreground (smica_planck,
source/CMBlikes.f90:1262-1339), one walker at a time, written from the reference
routines cited on each method.  Pinned against the compiled reference by
tests/golden/cmblikes_ref.json (oracle/gen_golden.py).  Only tests/ use it.

Matrix_Diagonalize (DSYEV) is numpy.linalg.eigh; Matrix_Inverse is
numpy.linalg.inv of the SPD covariance; sums follow the reference's loop
order where the order is visible in the source.
"""
from __future__ import annotations

import math
import os
import re

import numpy as np

CL_FIELDS = "TEBP"
T_CMB = 2.72548
H_PLANCK = 6.62606957e-34
K_B = 1.3806488e-23
GHZ_KELVIN = H_PLANCK / K_B * 1e9


class Ini:
    """Minimal IniObjects reader: key = value, first definition wins,
    INCLUDE()/DEFAULT(), overrides first (IniObjects.f90)."""

    def __init__(self, path, overrides=None):
        self.path = path
        self.kv = {}
        for k, v in (overrides or {}).items():
            self.kv[k] = str(v)
        self._read(path)

    def _read(self, path):
        with open(path) as f:
            for line in f:
                s = line.strip()
                if not s or s.startswith("#"):
                    continue
                m = re.match(r"^(INCLUDE|DEFAULT)\((.*)\)$", s, re.I)
                if m:
                    self._read(os.path.join(os.path.dirname(path), m.group(2).strip()))
                    continue
                if "=" not in s:
                    continue
                k, v = s.split("=", 1)
                k, v = k.strip(), v.strip()
                if k not in self.kv:
                    self.kv[k] = v

    def get(self, k, default=None):
        v = self.kv.get(k)
        return default if v is None or v == "" else v

    def fname(self, k, required=True):
        v = self.get(k)
        if v is None:
            if required:
                raise KeyError(k)
            return None
        return self.resolve(v)

    def resolve(self, v):
        if v.startswith("/"):
            return v
        cand = os.path.join(os.path.dirname(self.path), v)
        return cand if os.path.exists(cand) else v

    def logical(self, k, default):
        v = self.get(k)
        if v is None:
            return default
        return v.strip(".").upper()[0] in "TY1"


def _content_rows(path):
    rows = []
    with open(path) as f:
        for line in f:
            s = line.strip()
            if s and not s.startswith("#"):
                if "d" in s or "D" in s:
                    s = s.replace("d", "e").replace("D", "e")
                rows.append(np.array(s.split(), dtype=np.float64))
    return rows


def _last_top_comment(path):
    res = ""
    with open(path) as f:
        for line in f:
            if not line.strip():
                continue
            if line.startswith("#"):
                res = line[1:].strip()
            else:
                break
    return res


def _paramnames(path, derived=False):
    """ParamNames_Init (ObjectParamNames.f90:119-151): the non-derived names
    (DataParams); with derived=True also the '*' (derived) names."""
    names, dnames = [], []
    with open(path) as f:
        for line in f:
            t = line.split()
            if t and not t[0].startswith("#"):
                (dnames if t[0].endswith("*") else names).append(t[0].rstrip("*"))
    return (names, dnames) if derived else names


def _eigh(M):
    return np.linalg.eigh(M)


def _mat_root(M, pw):               # Matrix_Root (Matrix_utils_new.f90:421-440)
    d, U = _eigh(M)
    return (U * d ** pw) @ U.T


class CMBLikesOracle:
    """TCMBLikes / TBK_planck / TSmica_planck for one dataset;
    loglike(dl[10][lmax+1], nuis), derived(nuis)."""

    SMICA_PIVOT = 2000.0                                   # TSmica_planck%pivot (CMBlikes.f90:1270)

    def __init__(self, dataset, overrides=None, tag=""):
        ini = Ini(dataset, overrides)
        self.bk = tag == "BKPLANCK"
        self.smica = tag == "SMICA"
        # CMBLikes_ReadIni (CMBlikes.f90:466-749)
        s = ini.get("map_names")
        self.has_map_names = s is not None
        if self.has_map_names:
            self.map_names = s.split()
            self.map_fields = [CL_FIELDS.index(f[0]) + 1 for f in ini.get("map_fields").split()]
        else:
            self.map_names = list(CL_FIELDS)
            self.map_fields = [1, 2, 3, 4]
        s = ini.get("fields_use")
        use_field = [False] * 5
        if s:
            for f in s.split():
                use_field[CL_FIELDS.index(f[0]) + 1] = True
        else:
            use_field = [True] * 5
        nm = len(self.map_names)
        s = ini.get("maps_use")
        if s:
            use = [False] * nm
            for m in s.split():
                use[self.map_names.index(m)] = True
        else:
            use = [use_field[self.map_fields[i]] for i in range(nm)]
        req = list(use)
        s = ini.get("maps_required") if self.has_map_names else ini.get("fields_required")
        for m in (s or "").split():
            req[self.map_names.index(m)] = True
        self.like_approx = {"HL": 1, "gaussian": 2, "exact": 3}[ini.get("like_approx")]
        self.used_idx = [0] * nm
        self.req_idx = [0] * nm
        self.used_order, self.req_order = [], []
        for i in range(nm):
            if req[i]:
                self.req_order.append(i)
                self.req_idx[i] = len(self.req_order)
            if use[i]:
                self.used_order.append(self.map_names[i])
                self.used_idx[i] = len(self.used_order)
        self.nmaps = len(self.used_order)
        self.nreq = len(self.req_order)
        self.ncl = self.nmaps * (self.nmaps + 1) // 2
        self.lmin = int(ini.get("cl_lmin"))
        self.lmax = int(ini.get("cl_lmax"))
        self.binned = ini.logical("binned", False)
        self.aberration = float(ini.get("aberration_coeff", 0.0))
        if self.binned:
            self.nbins = int(ini.get("nbins", 0))
            self.bin_min = int(ini.get("use_min", 1))
            self.bin_max = int(ini.get("use_max", self.nbins))
        else:                                              # unbinned (:601-605, :636-637): bins are l
            self.nbins = self.lmax - self.lmin + 1
            self.bin_min = int(ini.get("use_min", self.lmin))
            self.bin_max = int(ini.get("use_max", self.lmax))
        self.bins = list(range(self.bin_min, self.bin_max + 1))
        if self.binned:
            self.W_main = self._read_windows(ini, "bin_window")
        self.clhat = self._read_cl(ini, "cl_hat")
        if self.like_approx == 1:
            self.clfid = self._read_cl(ini, "cl_fiducial")
        elif self.like_approx == 3:
            self.fksy = float(ini.get("fullsky_exact_fksy", 1.0))
        inc = ini.logical("cl_hat_includes_noise", False)
        self.clnoise = None
        if self.like_approx != 2 or inc:
            self.clnoise = self._read_cl(ini, "cl_noise")
            if not inc:
                self.clhat = {b: self.clhat[b] + self.clnoise[b] for b in self.bins}
            elif self.like_approx == 2:
                self.clhat = {b: self.clhat[b] - self.clnoise[b] for b in self.bins}
                self.clnoise = None
        fid_noise = ini.logical("cl_fiducial_includes_noise", False) if self.like_approx != 2 else False
        self.chatM, self.noiseM, self.sqrt_fid = {}, {}, {}
        for b in self.bins:
            self.chatM[b] = self._to_matrix(self.clhat[b])
            if self.clnoise is not None:
                self.noiseM[b] = self._to_matrix(self.clnoise[b])
            if self.like_approx == 1:
                f = self.clfid[b] + (0 if fid_noise else self.clnoise[b])
                self.sqrt_fid[b] = _mat_root(self._to_matrix(f), 0.5)
        if self.like_approx != 3:
            self._read_covmat(ini)
        self.fidcorr = None
        if ini.get("linear_correction_fiducial_file"):
            self.fidcorr = self._read_cl(ini, "linear_correction_fiducial")
            self.W_corr = self._read_windows(ini, "linear_correction_bin_window")
        self.cal_index = None
        self.log_cal_prior = -1.0
        cp = ini.fname("calibration_param", required=False)
        if cp:
            self.nuisance = _paramnames(cp)
            self.cal_index = len(self.nuisance) - 1
            self.log_cal_prior = float(ini.get("log_calibration_prior", -1.0))
        self.derived_names = []
        if self.smica:                                     # Tsmica_planck_ReadIni :1281-1293
            self.nuisance, self.derived_names = _paramnames(ini.fname("nuisance_params"), derived=True)
            cn = ini.get("calibration_paramname")
            if cn is not None:
                self.cal_index = self.nuisance.index(cn) if cn in self.nuisance else None
        if self.bk:
            self.nuisance = _paramnames(ini.fname("nuisance_params"))
            self.fpivot_dust = float(ini.get("fpivot_dust", 353.0))
            self.fpivot_sync = float(ini.get("fpivot_sync", 23.0))
            self.decorr_dust = [float(ini.get("fpivot_dust_decorr(1)", 217.0)),
                                float(ini.get("fpivot_dust_decorr(2)", 353.0))]
            self.decorr_sync = [float(ini.get("fpivot_sync_decorr(1)", 23.0)),
                                float(ini.get("fpivot_sync_decorr(2)", 33.0))]
            self.lform_dust = ini.get("lform_dust_decorr", "flat")
            self.lform_sync = ini.get("lform_sync_decorr", "flat")
            self.bandpasses = [self._read_bandpass(ini.fname(f"bandpass[{self.used_order[i]}]"))
                               for i in range(self.nreq)]

    # -- helpers restating the reference's index conventions
    def _cl_name(self, names, i, j):                       # Cl_i_j_name :328-343
        return names[i - 1] + ("x" if self.has_map_names else "") + names[j - 1]

    def _pair_indices(self, S, used_index):               # PairStringToUsedMapIndices :195-231
        if len(S) == 2 and not self.has_map_names:
            a, b = self.map_names.index(S[0]), self.map_names.index(S[1])
        else:
            x = S.index("x")
            a, b = self.map_names.index(S[:x]), self.map_names.index(S[x + 1:])
        i1, i2 = used_index[a], used_index[b]
        return (i1, i2) if i1 >= i2 else (i2, i1)

    def _cols(self, S):                                    # UseString_to_cols :234-260
        out = []
        for t in S.split():
            i1, i2 = self._pair_indices(t, self.used_idx)
            out.append(0 if (i1 == 0 or i2 == 0) else i1 * (i1 - 1) // 2 + i2)
        return out

    def _to_matrix(self, X):                               # ElementsToMatrix :950-965
        n = self.nmaps
        M = np.zeros((n, n))
        ix = 0
        for i in range(n):
            for j in range(i + 1):
                M[i, j] = M[j, i] = X[ix]
                ix += 1
        return M

    def _read_cl(self, ini, base):                         # ReadClArr :146-193
        fn = ini.fname(base + "_file")
        order = ini.get(base + "_order")
        incols = _last_top_comment(fn) if not order else "L " + order
        li = incols.split()
        cols = [0] * self.ncl
        ix = 0
        for i in range(1, self.nmaps + 1):
            for j in range(1, i + 1):
                nmij = self._cl_name(self.used_order, i, j)
                k = li.index(nmij) + 1 if nmij in li else -1
                if k == -1 and i != j:
                    nmji = self._cl_name(self.used_order, j, i)
                    k = li.index(nmji) + 1 if nmji in li else -1
                if k != -1:
                    cols[ix] = k
                ix += 1
        cl = {b: np.zeros(self.ncl) for b in self.bins}
        for r in _content_rows(fn):
            l = int(r[0])
            if self.bin_min <= l <= self.bin_max:
                for ix in range(self.ncl):
                    if cols[ix]:
                        cl[l][ix] = r[cols[ix] - 1]
        return cl

    def _read_windows(self, ini, t):                       # ReadBinWindows :371-414
        fname = ini.get(t + "_files")
        o1 = ini.get(t + "_in_order")
        o2 = ini.get(t + "_out_order", o1)
        cin = [self._pair_indices(s, self.req_idx) for s in o1.split()]
        cout = self._cols(o2)
        L = self.lmax - self.lmin + 1
        W = {}
        for b in self.bins:
            Wb = np.zeros((len(cin), L))
            for r in _content_rows(ini.resolve(fname.replace("%u", str(b)))):
                l = int(r[0])
                if self.lmin <= l <= self.lmax:
                    Wb[:, l - self.lmin] = r[1:1 + len(cin)]
            W[b] = Wb
        return {"in": cin, "out": cout, "W": W}

    def _read_covmat(self, ini):                           # ReadCovmat :752-795
        cl_in = self._cols(ini.get("covmat_cl"))
        self.cl_use = [c for c in cl_in if c]
        used = [i for i, c in enumerate(cl_in) if c]
        nin = len(cl_in)
        cov = np.concatenate(_content_rows(ini.fname("covmat_fiducial"))).reshape(nin * self.nbins,
                                                                                  nin * self.nbins)
        scale = float(ini.get("covmat_scale", 1.0))
        nu = len(self.cl_use)
        nb = len(self.bins)
        C = np.zeros((nb * nu, nb * nu))
        used = np.array(used)
        for bx in self.bins:
            for by in self.bins:
                C[(bx - self.bin_min) * nu:(bx - self.bin_min + 1) * nu, (by - self.bin_min) * nu:(by - self.bin_min + 1) * nu] = \
                    scale * cov[np.ix_((bx - 1) * nin + used, (by - 1) * nin + used)]
        self.inv_cov = np.linalg.inv(C)

    def _read_bandpass(self, fn):                          # TBK_planck_Read_Bandpass :72-105
        R = np.array(_content_rows(fn))
        nu, tr = R[:, 0], R[:, 1]
        n = len(nu)
        dnu = np.empty(n)
        dnu[0] = nu[1] - nu[0]
        dnu[1:-1] = (nu[2:] - nu[:-2]) / 2
        dnu[-1] = nu[-1] - nu[-2]
        e = np.exp(GHZ_KELVIN * nu / T_CMB)
        th_int = np.sum(dnu * tr * nu ** 4 * e / (e - 1) ** 2)

        def th0(nu0):
            e0 = np.exp(GHZ_KELVIN * nu0 / T_CMB)
            return nu0 ** 4 * e0 / (e0 - 1) ** 2
        return {"nu": nu, "R": tr, "dnu": dnu, "th_dust": th_int / th0(self.fpivot_dust),
                "th_sync": th_int / th0(self.fpivot_sync), "nu_bar": np.sum(dnu * nu * tr) / np.sum(dnu * tr)}

    # -- the likelihood
    def _theory_field(self, dl, i, j):
        f1 = self.map_fields[self.req_order[i - 1]]
        f2 = self.map_fields[self.req_order[j - 1]]
        if f2 > f1:
            f1, f2 = f2, f1
        return f1, f2, dl[f1 * (f1 - 1) // 2 + f2 - 1]

    def map_cls(self, dl, nuis):
        """GetTheoryMapCls + AdaptTheoryForMaps (CMBlikes.f90:1022-1126)."""
        lo, hi = self.lmin, self.lmax
        ells = np.arange(lo, hi + 1, dtype=np.float64)
        C = {}
        for i in range(1, self.nreq + 1):
            for j in range(1, i + 1):
                f1, f2, th = self._theory_field(dl, i, j)
                C[i, j] = (f1, f2, np.array(th[lo:hi + 1], dtype=np.float64))
        if self.aberration != 0:                           # AddAberration :1062-1101
            for k, (f1, f2, cl) in C.items():
                if f1 <= 3 and f2 <= 3:
                    d = cl / (ells * (ells + 1))
                    dd = d.copy()
                    dd[1:-1] = 0.5 * (d[2:] - d[:-2])
                    dd[0] = dd[1]
                    dd[-1] = dd[-2]
                    dd = ells ** 2 * (ells + 1) * dd
                    C[k] = (f1, f2, cl + self.aberration * dd)
        if self.bk:
            self._add_foregrounds(C, nuis)
        if self.smica:
            self._add_smica_foregrounds(C, nuis, ells)
        if self.cal_index is not None:
            cal = nuis[self.cal_index]
            for k, (f1, f2, cl) in C.items():
                if f1 <= 3 and f2 <= 3:
                    C[k] = (f1, f2, cl / cal ** 2)
        return {k: v[2] for k, v in C.items()}

    def _smica_fg(self, P, ells):                          # TSmica_planck_AddForegrounds :1303-1317
        A1, n1, n1run, A2, n2 = P[:5]
        out1 = np.empty(ells.size)
        out2 = np.empty(ells.size)
        for k, l in enumerate(ells):                       # scalar libm, one l at a time
            lnrat = math.log(l / self.SMICA_PIVOT)
            out1[k] = A1 * math.exp(n1 * lnrat + n1run / 2 * lnrat ** 2)
            out2[k] = A2 * (l / self.SMICA_PIVOT) ** n2
        return out1, out2

    def _add_smica_foregrounds(self, C, P, ells):
        t1, t2 = self._smica_fg(P, ells)
        for k, (f1, f2, cl) in C.items():
            if f1 == 1 and f2 == 1:                        # CL%theory_i == 1 .and. CL%theory_j == 1
                C[k] = (f1, f2, (cl + t1) + t2)

    def derived(self, nuis):
        """derivedParameters (TSmica_planck_derivedParameters :1324-1337; the base
        TDataLikelihood_derivedParameters is zeros, GeneralTypes.f90:504-512)."""
        out = np.zeros(len(self.derived_names))
        if self.smica and out.size:
            f1, f2, _ = self._theory_field(np.zeros((10, self.lmax + 1)), 1, 1)
            if f1 == 1 and f2 == 1:
                t1, t2 = self._smica_fg(nuis, np.array([2000.0]))
                out[0] = (0.0 + t1[0]) + t2[0]
        return out

    def _add_foregrounds(self, C, P):                      # TBK_planck_AddForegrounds :229-340
        Adust, Async, alphadust, betadust, Tdust, alphasync, betasync, corr = P[:8]
        EEd, EEs, Dd, Ds = P[8:12]
        fd, fs, bc = [], [], []
        for i in range(self.nreq):
            nm = self.used_order[i]
            if "95" in nm:
                b = P[12] + P[13] + 1.
            elif "150" in nm:
                b = P[12] + P[14] + 1.
            elif "220" in nm:
                b = P[12] + P[15] + 1.
            else:
                b = 1.
            bp = self.bandpasses[i]
            nu, R, dnu = bp["nu"], bp["R"], bp["dnu"]
            gb = np.sum(dnu * R * nu ** (3 + betadust) / (np.exp(GHZ_KELVIN * nu / Tdust) - 1))
            gb0 = self.fpivot_dust ** (3 + betadust) / (np.exp(GHZ_KELVIN * self.fpivot_dust / Tdust) - 1)
            pl = np.sum(dnu * R * nu ** (2 + betasync))
            pl0 = self.fpivot_sync ** (2 + betasync)
            if b != 1.:
                nb_ = bp["nu_bar"]
                th_err = b ** 4 * np.exp(GHZ_KELVIN * nb_ * (b - 1) / T_CMB) * \
                    (np.exp(GHZ_KELVIN * nb_ / T_CMB) - 1) ** 2 / (np.exp(GHZ_KELVIN * nb_ * b / T_CMB) - 1) ** 2
                gb_err = b ** (3 + betadust) * (np.exp(GHZ_KELVIN * nb_ / Tdust) - 1) / \
                    (np.exp(GHZ_KELVIN * nb_ * b / Tdust) - 1)
                pl_err = b ** (2 + betasync)
            else:
                th_err = gb_err = pl_err = 1.0
            fd.append((gb / gb0) / bp["th_dust"] * (gb_err / th_err))
            fs.append((pl / pl0) / bp["th_sync"] * (pl_err / th_err))
            bc.append(b)
        ells = np.arange(self.lmin, self.lmax + 1, dtype=np.float64)
        dustpow = Adust * (ells / 80.0) ** alphadust
        syncpow = Async * (ells / 80.0) ** alphasync
        dspow = corr * np.sqrt(Adust * Async) * (ells / 80.0) ** ((alphadust + alphasync) / 2)
        need_d, need_s = abs(Dd - 1) > 1e-5, abs(Ds - 1) > 1e-5

        def decorr(Delta, nu0, nu1, piv, lform):        # Decorrelation :187-227
            scl_nu = np.log(nu0 / nu1) ** 2 / np.log(piv[0] / piv[1]) ** 2
            scl_ell = {"lin": ells / 80.0, "quad": (ells / 80.0) ** 2}.get(lform, np.ones_like(ells))
            if Delta > 1:
                return 2.0 - np.exp(np.log(2.0 - Delta) * scl_nu * scl_ell)
            return np.exp(np.log(Delta) * scl_nu * scl_ell)
        for (i, j), (f1, f2, cl) in list(C.items()):
            if not ((f1 == 2 and f2 == 2) or (f1 == 3 and f2 == 3)):
                continue
            a, b = i - 1, j - 1
            dust = fd[a] * fd[b]
            sync = fs[a] * fs[b]
            ds = fd[a] * fs[b] + fs[a] * fd[b]
            if f1 == 2:
                dust *= EEd
                sync *= EEs
                ds *= np.sqrt(EEd * EEs)
            nua, nub = self.bandpasses[a]["nu_bar"] * bc[a], self.bandpasses[b]["nu_bar"] * bc[b]
            Dpd = decorr(Dd, nua, nub, self.decorr_dust, self.lform_dust) if (need_d and i != j) else 1.0
            Dps = decorr(Ds, nua, nub, self.decorr_sync, self.lform_sync) if (need_s and i != j) else 1.0
            C[i, j] = (f1, f2, cl + dust * dustpow * Dpd + sync * syncpow * Dps + ds * dspow)

    def _bin(self, win, mc, b):                            # TBinWindows_bin :1230-1256
        cls = np.zeros(self.ncl)
        for k, ((i1, i2), out) in enumerate(zip(win["in"], win["out"])):
            if out > 0:
                cls[out - 1] += np.dot(win["W"][b][k], mc[i1, i2])
        return cls

    def _transform(self, C, Chat, CfHalf):                 # CMBLikes_Transform :861-914
        d, U = _eigh(C)
        rot = U.T @ Chat @ U
        roots = np.sqrt(d)
        rot = rot / roots[:, None] / roots[None, :]
        rot = U @ rot @ U.T
        d2, V = _eigh(rot)
        g = np.sign(d2 - 1) * np.sqrt(2 * np.maximum(0, d2 - np.log(d2) - 1))
        U2 = CfHalf @ V
        return (U2 * g) @ U2.T

    def _exact_chisq(self, C, Chat, l):                  # ExactChiSq :967-979
        R = _mat_root(C, -0.5)
        M = R @ (Chat @ R)
        L = np.linalg.cholesky(M)                          # MatrixSym_LogDet (Matrix_utils_new.f90:619-634)
        logdet = 2.0 * np.sum(np.log(np.diag(L)))
        return (2 * l + 1) * self.fksy * (np.trace(M) - self.nmaps - logdet)

    def loglike(self, dl, nuis):
        """-lnL (CMBLikes_LogLike, CMBlikes.f90:1165-1227)."""
        mc = self.map_cls(dl, nuis)
        if self.like_approx == 3:                          # unbinned exact (:1187-1206)
            chisq = 0.0
            for l in self.bins:
                C = np.zeros((self.nmaps, self.nmaps))
                for i in range(1, self.nmaps + 1):
                    for j in range(1, i + 1):
                        C[i - 1, j - 1] = C[j - 1, i - 1] = mc[i, j][l - self.lmin]
                C = C + self.noiseM[l]
                chisq += self._exact_chisq(C, self.chatM[l], l)
            if self.log_cal_prior > 0 and self.cal_index is not None:
                chisq += (np.log(nuis[self.cal_index]) / self.log_cal_prior) ** 2
            return chisq / 2
        X = []
        for b in self.bins:
            cls = self._bin(self.W_main, mc, b)
            if self.fidcorr is not None:
                cls = cls + (self._bin(self.W_corr, mc, b) - self.fidcorr[b])
            C = self._to_matrix(cls)
            if self.noiseM:
                C = C + self.noiseM[b]
            if self.like_approx == 1:
                M = self._transform(C, self.chatM[b], self.sqrt_fid[b])
            else:
                M = C - self.chatM[b]
            vec = np.array([M[i, j] for i in range(self.nmaps) for j in range(i + 1)])
            X.extend(vec[np.array(self.cl_use) - 1])
        X = np.array(X)
        chisq = X @ self.inv_cov @ X
        if self.log_cal_prior > 0 and self.cal_index is not None:
            chisq += (np.log(nuis[self.cal_index]) / self.log_cal_prior) ** 2
        return chisq / 2
