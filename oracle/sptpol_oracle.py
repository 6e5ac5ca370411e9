"""ORACLE TEST INFRASTRUCTURE -- never imported by the product path.

numpy restatement of the SPTpol bandpower likelihoods of the reference:

  TSPTpolEELike  source/CMB_SPTpol_TEEE_2017.f90
      SPTpol_TEEE_ReadIni            :56-140   (ini keys, priors; Read_Real is REAL(4))
      InitSPTpolData                 :142-352  (desc, bandpowers, cov, windows, beam)
      SPTpolEELnLike                 :356-567
  TSPTpolBBLike  source/CMB_SPTpol_BB_2019.f90
      SPTpol_BB_ReadIni              :56-147
      InitSPTpolBBData               :149-438
      SPTpolBBLnLike                 :441-656
      dBdT / Bnu / dustFreqScalingFrom150GHz :750-815
  Matrix_CholeskyDouble / Matrix_GaussianLogLikeCholDouble (module-local copies,
      TEEE :614-665, BB :722-745): dpotrf 'L', log det = sum log L_ii,
      chi^2/2 = d . (C^-1 d) / 2 via dpotrs.

Single-precision literals of the reference (REAL(4) constants promoted to
double, e.g. ``beta = 1.59``, ``hk = 4.799237e-2``, ``x0 = nu0/56.78``, the
``**1.42`` exponent) are reproduced with np.float32(...) so the arithmetic is
the reference's.  Pinned against the compiled reference in
tests/golden/sptpol_ref.json (oracle/gen_golden.py ``sptpol``).
"""
from __future__ import annotations

import os

import numpy as np
from scipy.linalg import cho_solve

TWOPI = 6.283185307179586476925286766559
F = lambda x: float(np.float32(x))          # noqa: E731  REAL(4) literal / Ini%Read_Real


def _ini(path: str, overrides: dict | None = None) -> dict:
    kv = {}
    for k, v in (overrides or {}).items():
        kv[k] = str(v)
    with open(path) as f:
        for line in f:
            s = line.strip()
            if not s or s.startswith("#") or "=" not in s:
                continue
            k, v = s.split("=", 1)
            kv.setdefault(k.strip(), v.strip())
    return kv


def _logical(kv, key, default=False):
    v = kv.get(key, "")
    if v == "":
        return default
    return v.strip().upper().lstrip(".").startswith("T")


def _real(kv, key, default):
    """Ini%Read_Real: a REAL(4) value (default or parsed)."""
    v = kv.get(key, "")
    return F(float(v) if v != "" else default)


def _n_params(path: str) -> int:
    n = 0
    with open(path) as f:
        for line in f:
            s = line.strip()
            if s and not s.startswith("#"):
                n += 1
    return n


def _chol(cov):
    return np.linalg.cholesky(cov)       # dpotrf 'L'


def _gauss_loglike_chol(L, d):
    """Matrix_GaussianLogLikeCholDouble: sum log L_ii + d.(C^-1 d)/2."""
    ld = float(np.sum(np.log(np.diag(L))))
    tmp = cho_solve((L, True), d)
    return ld + float(np.dot(tmp, d)) / 2.0


class SptpolTEEE:
    def __init__(self, dataset: str, overrides: dict | None = None):
        kv = _ini(dataset, overrides)
        self.EEonly = _logical(kv, "sptpol_EEonly")
        self.TEonly = _logical(kv, "sptpol_TEonly")
        self.aberration = _logical(kv, "correct_aberration")
        self.Tcal_prior = _logical(kv, "sptpol_tcal_prior")
        self.meanTcal = _real(kv, "sptpol_meanTcal", 1.0)
        self.sigmaTcal = np.log(1 + _real(kv, "sptpol_sigmaTcal", 0.005))
        self.Pcal_prior = _logical(kv, "sptpol_pcal_prior")
        self.meanPcal = _real(kv, "sptpol_meanPcal", 1.0)
        _real(kv, "sptpol_sigmaPcal", 0.02)
        self.sigmaPcal = np.log(1 + self.sigmaTcal)          # :79 (sic: uses sigmaTcal)
        self.kappa_prior = _logical(kv, "sptpol_kappa_prior")
        self.meankappa = _real(kv, "sptpol_meankappa", 0.0)
        self.sigmakappa = _real(kv, "sptpol_sigmakappa", 0.001)
        self.aEE_prior = _logical(kv, "sptpol_alphaEE_prior")
        self.meanAlphaEE = _real(kv, "sptpol_meanAlphaEE", -2.42)
        self.sigmaAlphaEE = _real(kv, "sptpol_sigmaAlphaEE", 0.02)
        self.aTE_prior = _logical(kv, "sptpol_alphaTE_prior")
        self.meanAlphaTE = _real(kv, "sptpol_meanAlphaTE", -2.42)
        self.sigmaAlphaTE = _real(kv, "sptpol_sigmaAlphaTE", 0.02)
        self.n_nuis = _n_params(kv["sptpol_TEEE_params_file"])
        with open(kv["sptpol_TEEE_desc_file"]) as f:
            toks = f.read().split()
        nbin, nfreq, lmin, lmax = (int(t) for t in toks[:4])
        self.nbin, self.lmin, self.lmax = nbin, lmin, lmax
        nall = 2 * nbin
        bp = np.loadtxt(kv["sptpol_TEEE_bp_file"], ndmin=2)
        self.spec = bp[:3 * nbin, 1].reshape(3, nbin)
        cov = np.fromfile(kv["sptpol_TEEE_cov_file"], dtype="<f8", count=nall * nall).reshape(nall, nall).T.copy()
        if self.EEonly or self.TEonly:                      # :243-262
            cov[:nbin, nbin:] *= 1e12
            cov[nbin:, :nbin] *= 1e12
            if self.EEonly:
                cov[:nbin, :nbin] *= 1e24
            if self.TEonly:
                cov[nbin:, nbin:] *= 1e24
        self.L = _chol(cov)
        wd = kv["sptpol_TEEE_window_dir"]
        self.windows = np.zeros((lmax - lmin + 1, nall))
        for i in range(nall):
            w = np.loadtxt(wd + f"window_{i + 1}", ndmin=2)
            self.windows[:, i] = w[:lmax - lmin + 1, 1]
        be = np.loadtxt(kv["sptpol_TEEE_beam_file"], ndmin=2)[:, 1]
        self.beam_err = be[:2 * nall].reshape(2, nall)       # [term][bandpower]
        ells = np.arange(lmin - 1, lmax + 2, dtype=np.float64)
        self.ells = ells
        self.conv = (ells * (ells + 1.0)) / TWOPI
        self.rawspec = ells ** 3 / self.conv
        self.deriv_factor = 0.5 / ells[1:-1] ** 2

    def loglike(self, dl: np.ndarray, P: np.ndarray) -> float:
        """dl: [n_fields >= 3, l] D_l from l = 0 (TT, TE, EE ...); P: DataParams."""
        lmin, lmax, nbin = self.lmin, self.lmax, self.nbin
        d3000 = 3000 * 3001 / TWOPI
        beta, dcos = F(0.0012309), F(-0.4033)
        tmp2 = np.zeros(2 * nbin)
        pois = P[1:3] / d3000
        adust = (P[3], P[5])
        alpha = (P[4], P[6])
        cal = [(P[7] * P[7]) * P[8] ** i for i in range(3)]
        L = np.arange(lmin, lmax + 1, dtype=np.float64)
        for k in range(2):
            field = (1, 2)[k]
            d = np.zeros(lmax + 2)
            n = min(lmax + 1, dl.shape[1] - 1)
            d[1:n + 1] = dl[field, 1:n + 1]                   # ClArray: cl(1:lmax+1)
            dls = d[lmin - 1:lmax + 2]
            raw = self.rawspec * dls
            deriv = self.deriv_factor * (raw[2:] - raw[:-2])
            ab = np.zeros(L.size)
            if self.aberration:
                ab = (d[lmin + 1:lmax + 2] - d[lmin - 1:lmax]) / 2.0
                ab = (-1 * beta * dcos) * L * ab
            fg = (pois[k] - P[0] * deriv) * self.conv[1:-1]
            fg = fg + d[lmin:lmax + 1]
            fg = fg + ab
            fg = fg + adust[k] * (L / 80.0) ** (alpha[k] + 2.0)
            tmp = self.windows[:, k * nbin:(k + 1) * nbin].T @ fg
            tmp2[k * nbin:(k + 1) * nbin] = tmp / cal[k + 1]
        bf = np.ones(2 * nbin)
        for t in range(2):
            bf = bf * (1 + self.beam_err[t] * P[9 + t])
        delta = tmp2 * bf
        delta[:nbin] -= self.spec[0]
        delta[nbin:] -= self.spec[1]
        lnl = _gauss_loglike_chol(self.L, delta)
        prior = 0.5 * float(np.sum(P[9:11] ** 2))
        if self.Tcal_prior:
            prior += 0.5 * (np.log(P[7] / self.meanTcal) / self.sigmaTcal) ** 2
        if self.Pcal_prior:
            prior += 0.5 * (np.log(P[8] / self.meanPcal) / self.sigmaPcal) ** 2
        if self.kappa_prior:
            prior += 0.5 * ((P[0] - self.meankappa) / self.sigmakappa) ** 2
        if self.aTE_prior:
            prior += 0.5 * ((P[4] - self.meanAlphaTE) / self.sigmaAlphaTE) ** 2
        if self.aEE_prior:
            prior += 0.5 * ((P[6] - self.meanAlphaEE) / self.sigmaAlphaEE) ** 2
        return lnl + prior

    def loglike_batch(self, dl: np.ndarray, nuis: np.ndarray) -> np.ndarray:
        return np.array([self.loglike(dl[w], nuis[w]) for w in range(dl.shape[0])])


def _dBdT(nu, nu0):
    x0 = nu0 / F(56.78)
    dBdT0 = x0 ** 4 * np.exp(x0) / (np.exp(x0) - 1) ** 2
    x = nu / F(56.78)
    return x ** 4 * np.exp(x) / (np.exp(x) - 1) ** 2 / dBdT0


def _Bnu(nu, nu0, T):
    hk = F(4.799237e-2)
    b = (nu / nu0) ** 3
    return b * (np.exp(hk * nu0 / T) - 1.0) / (np.exp(hk * nu / T) - 1.0)


def dust_scaling_from_150(f1, f2):
    beta, Tdust = F(1.59), F(19.6)
    s = ((f1 * f2) / (150.0 * 150.0)) ** beta
    s = s * _Bnu(f1, 150.0, Tdust) * _Bnu(f2, 150.0, Tdust)
    return s / _dBdT(f1, 150.0) / _dBdT(f2, 150.0)


class SptpolBB:
    def __init__(self, dataset: str, overrides: dict | None = None):
        kv = _ini(dataset, overrides)
        self.blind_abb = 0.0
        drop = [_logical(kv, "sptpol_drop_150x150ghz"), _logical(kv, "sptpol_drop_90x150ghz"),
                _logical(kv, "sptpol_drop_90x90ghz")]
        self.cal_prior = _logical(kv, "sptpol_cal_prior")
        self.icc = np.array([[_real(kv, "sptpol_invCal_90x90", 0.0004), _real(kv, "sptpol_invCal_90x150", 0.0)],
                             [0.0, _real(kv, "sptpol_invCal_150x150", 0.0004)]])
        self.icc[1, 0] = self.icc[0, 1]
        self.add_prior = _logical(kv, "sptpol_Add_prior")
        self.meanAdd = _real(kv, "sptpol_meanAdd", 0.0132)
        self.sigmaAdd = _real(kv, "sptpol_sigmaAdd", 0.0055)
        self.n_nuis = _n_params(kv["sptpol_BB_params_file"])
        with open(kv["sptpol_BB_desc_file"]) as f:
            toks = f.read().split()
        nbin, nfreq, lmin, lmax = (int(t) for t in toks[:4])
        eff = [float(t) for t in toks[4:4 + nfreq]]
        self.nbin, self.lmin, self.lmax = nbin, lmin, lmax
        nall = 3 * nbin
        pairs = [(eff[i], eff[j]) for i in range(nfreq) for j in range(i, nfreq)]
        self.dust_scale = [dust_scaling_from_150(a, b) for a, b in pairs]
        ells = np.arange(lmin, lmax + 1, dtype=np.float64)
        self.ells = ells
        self.poisson = (ells * (ells + 1.0)) / (3000.0 * 3001.0)
        self.galdust = ((ells + 1.0) / 81.0) * (80.0 / ells) ** F(1.42)
        spec = np.zeros((3, nbin))
        k = 0
        with open(kv["sptpol_BB_bp_file"]) as f:
            for line in f:
                s = line.strip()
                if k >= nbin:
                    break
                if s.find("#") + s.find("!") + 2 == 1:       # index('#')+index('!') == 1
                    continue
                v = s.split()
                spec[0, k], spec[1, k], spec[2, k] = float(v[5]), float(v[4]), float(v[3])
                k += 1
        self.spec = spec
        cov = np.fromfile(kv["sptpol_BB_cov_file"], dtype="<f8", count=nall * nall).reshape(nall, nall).T.copy()
        for band in range(3):
            if drop[band]:
                for i in range(nbin):
                    t = band * nbin + i
                    tmp = cov[t, t]
                    cov[t, :] = 0
                    cov[:, t] = 0
                    cov[t, t] = 1e12 * tmp
        self.L = _chol(cov)
        raw = np.fromfile(kv["sptpol_BB_window_file"], dtype="<u1")
        i0, i1 = np.frombuffer(raw[:8].tobytes(), dtype="<i4")
        assert i0 == lmin and i1 == lmax
        self.windows = np.frombuffer(raw[8:8 + 8 * (lmax - lmin + 1) * nall].tobytes(), dtype="<f8").reshape(
            nall, lmax - lmin + 1).T
        rb = np.fromfile(kv["sptpol_BB_beam_file"], dtype="<u1")
        neff, nterm = np.frombuffer(rb[:8].tobytes(), dtype="<i4")
        self.beam_err = np.frombuffer(rb[8:8 + 8 * neff * nterm].tobytes(), dtype="<f8").reshape(nterm, neff)
        if _logical(kv, "sptpol_blind_abb"):
            self.blind_abb = float(np.fromfile(kv["sptpol_blind_abb_file"], dtype="<f8", count=1)[0])
        self.tensor = np.zeros(ells.size)
        rt = kv.get("r_template_file", "")
        if rt:
            with open(rt) as f:
                for line in f:
                    s = line.strip()
                    if not s or s.find("#") + s.find("!") + 2 == 1:
                        continue
                    v = s.split()
                    l = int(v[0])
                    if lmin <= l <= lmax:
                        self.tensor[l - lmin] = float(v[3])

    def loglike(self, dl: np.ndarray, P: np.ndarray) -> float:
        lmin, lmax, nbin = self.lmin, self.lmax, self.nbin
        d = np.zeros(lmax + 2)
        n = min(lmax + 1, dl.shape[1] - 1)
        d[1:n + 1] = dl[5, 1:n + 1]
        if P[0] != 1:
            d = d * (P[0] + self.blind_abb)
        if P[0] == 0:
            d[:] = 0
        d = d + P[2]
        d[lmin:lmax + 1] = d[lmin:lmax + 1] + P[1] * self.tensor
        pois = P[4:7]
        dust150 = P[3] * self.galdust
        cal = [P[7] * P[7], P[8] * P[7], P[8] * P[8]]
        tmp2 = np.zeros(3 * nbin)
        for k in range(3):
            fg = pois[k] * self.poisson
            fg = fg + dust150 * self.dust_scale[k]
            fg = fg + d[lmin:lmax + 1]
            tmp = self.windows[:, k * nbin:(k + 1) * nbin].T @ fg
            tmp2[k * nbin:(k + 1) * nbin] = tmp / cal[k]
        bf = np.ones(3 * nbin)
        for t in range(self.beam_err.shape[0]):
            bf = bf * (1 + self.beam_err[t] * P[9 + t])
        delta = tmp2 * bf
        for k in range(3):
            delta[k * nbin:(k + 1) * nbin] -= self.spec[k]
        lnl = _gauss_loglike_chol(self.L, delta)
        prior = 0.5 * float(np.sum(P[9:16] ** 2))
        if self.cal_prior:
            y1, y2 = np.log(P[8]), np.log(P[7])
            prior += 0.5 * (self.icc[0, 0] * y1 * y1 + 2 * self.icc[0, 1] * y1 * y2 + self.icc[1, 1] * y2 * y2)
        if self.add_prior:
            prior += 0.5 * ((P[3] - self.meanAdd) / self.sigmaAdd) ** 2
        return lnl + prior

    def loglike_batch(self, dl: np.ndarray, nuis: np.ndarray) -> np.ndarray:
        return np.array([self.loglike(dl[w], nuis[w]) for w in range(dl.shape[0])])


def open_sptpol(tag: str, dataset: str, overrides: dict | None = None):
    return (SptpolTEEE if tag == "SPTPOL_TEEE" else SptpolBB)(dataset, overrides)


__all__ = ["SptpolTEEE", "SptpolBB", "open_sptpol", "dust_scaling_from_150", "os"]
