"""Deterministic synthetic inputs for the plik_lite fast-parameter path.

The real plik_lite dataset (``plik_lite_v18_*.clik`` or a native ``.dataset``)
is not shipped with the reference (``.MISSING_LARGE_BLOBS``), so the parity
tests, the oracle harness and ``bench.py`` all build the same synthetic dataset
from a seed, exactly as SURVEY.md section 8(d) specifies:

* bins: widths 5x14, 9x156, 17x30, 33x15 starting at l=30 (TT 215 bins to
  l=2508; TE/EE use the first 199 bins, to l=1996) -- the layout of
  ``TPlikLiteLikelihood`` (reference ``source/CMB.f90:33-36``);
* ``weights`` file = 1/width per l (the reader multiplies by 2pi/(l(l+1)),
  ``source/CMB.f90:230-233``);
* ``X`` = binned best-fit theory x (1 + 0.01 N(0,1));
* ``cov`` = D (I + 0.05 A A^T / N_b) D with sigma_b = 2% |X_b| (floored at
  10% of the spectrum's rms |X| so TE zero crossings stay well conditioned),
  A ~ N(0,1);
* per-walker theory ``D_l (1 + 0.01 s_w(l))`` with ``s_w`` five cosine modes;
* ``calPlanck ~ N(1, 0.0025)`` (``batch2/planck_calibration.ini:2``).

Random numbers come from a counter-based splitmix64 stream + Box-Muller so
the same arrays are reproduced bit-for-bit on any host (numpy only, no
numpy.random version dependence).
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
_GOLDEN = np.uint64(0x9E3779B97F4A7C15)

PLMIN = 30
PLMAX = 2508
NBINCL = (215, 199, 199)          # TT, TE, EE  (source/CMB.f90:36)
BIN_WIDTHS = ((5, 14), (9, 156), (17, 30), (33, 15))

# field-pair index of Theory%Cls(i,j), i>=j, T=1 E=2 B=3 P=4 (CosmologyTypes.f90:24)
FIELD_TT, FIELD_TE, FIELD_EE, FIELD_BT, FIELD_BE, FIELD_BB = 0, 1, 2, 3, 4, 5
FIELD_PT, FIELD_PE, FIELD_PB, FIELD_PP = 6, 7, 8, 9
N_FIELDS = 10


def splitmix64(seed: int, n: int, offset: int = 0) -> np.ndarray:
    """n outputs of the splitmix64 stream for ``seed`` starting at ``offset``."""
    with np.errstate(over="ignore"):
        i = np.arange(offset + 1, offset + n + 1, dtype=np.uint64)
        z = (np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + i * _GOLDEN) & _M64
        z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & _M64
        z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & _M64
        z = z ^ (z >> np.uint64(31))
    return z


def uniforms(seed: int, n: int, offset: int = 0) -> np.ndarray:
    """Uniform doubles in [0, 1) with 53 random bits."""
    return (splitmix64(seed, n, offset) >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)


def gaussians(seed: int, n: int) -> np.ndarray:
    """n standard normals (Box-Muller, cosine branch; two uniforms each)."""
    u = uniforms(seed, 2 * n)
    u1 = 1.0 - u[0::2]          # (0, 1]
    u2 = u[1::2]
    return np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)


def _golden_dir() -> str:
    return os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")


def base_theory(lmax: int = PLMAX) -> np.ndarray:
    """Best-fit D_l (muK^2) for the 10 field pairs, shape [10, lmax+1], l=0..lmax.

    Source: ``data/base_plikHM_TTTEEE_lowl_lowE.minimum.theory_cl`` of the
    reference (columns TT TE EE BB PP, l=2..2508), stored as a fixture.
    """
    z = np.load(os.path.join(_golden_dir(), "base_plikHM_TTTEEE_lowl_lowE.theory_cl.npz"))
    L = z["L"]
    out = np.zeros((N_FIELDS, lmax + 1))
    m = L <= lmax
    for f, key in ((FIELD_TT, "TT"), (FIELD_TE, "TE"), (FIELD_EE, "EE"), (FIELD_BB, "BB"), (FIELD_PP, "PP")):
        out[f, L[m]] = z[key][m]
        if lmax > L[-1]:
            # beyond the file (l > 2508, e.g. SPT-SZ to 3300): damping-tail
            # extrapolation D_l = D_2508 exp(-(l - 2508) / 600), (2508/l)^2 for PP
            ell = np.arange(L[-1] + 1, lmax + 1, dtype=np.float64)
            tail = (L[-1] / ell) ** 2 if key == "PP" else np.exp(-(ell - L[-1]) / 600.0)
            out[f, L[-1] + 1:] = z[key][-1] * tail
    return out


def plik_bins() -> tuple[np.ndarray, np.ndarray]:
    """blmin/blmax as 0-based offsets from PLMIN (the on-disk convention, CMB.f90:224-227)."""
    lo, hi = [], []
    l = 0
    for w, n in BIN_WIDTHS:
        for _ in range(n):
            lo.append(l)
            hi.append(l + w - 1)
            l += w
    assert l == PLMAX - PLMIN + 1 and len(lo) == NBINCL[0]
    return np.array(lo, dtype=np.int64), np.array(hi, dtype=np.int64)


@dataclass
class PlikLiteData:
    """Synthetic plik_lite dataset in the on-disk form read by CMB.f90:208-303."""
    blmin: np.ndarray      # [215] offsets from PLMIN
    blmax: np.ndarray      # [215]
    weights_file: np.ndarray  # [2479] raw weights (before the 2pi/(l(l+1)) factor)
    X: np.ndarray          # [613] bandpowers (C_l units), TT|TE|EE
    cov: np.ndarray        # [613, 613]

    def internal_weights(self) -> np.ndarray:
        """Weights as used in LogLike: w_l * 2pi/(l(l+1)), index 0 <-> l=PLMIN."""
        ls = PLMIN + np.arange(self.weights_file.size, dtype=np.float64)
        return self.weights_file * (2.0 * np.pi) / ls / (ls + 1.0)

    def write(self, directory: str, name: str = "plik_lite_synth", use_cl: str = "TT TE EE",
              extra: dict | None = None) -> str:
        """Write the dataset files + a CosmoMC ``.dataset`` ini; return its path."""
        os.makedirs(directory, exist_ok=True)
        np.savetxt(os.path.join(directory, f"{name}_bins_min.txt"), self.blmin, fmt="%d")
        np.savetxt(os.path.join(directory, f"{name}_bins_max.txt"), self.blmax, fmt="%d")
        np.savetxt(os.path.join(directory, f"{name}_weights.txt"), self.weights_file, fmt="%.17e")
        nb = self.X.size
        np.savetxt(os.path.join(directory, f"{name}_data.txt"),
                   np.column_stack([np.arange(1, nb + 1), self.X]), fmt=["%d", "%.17e"])
        np.savetxt(os.path.join(directory, f"{name}_cov.txt"), self.cov, fmt="%.17e")
        with open(os.path.join(directory, "planck_calib.paramnames"), "w") as f:
            f.write("calPlanck     y_{\\rm cal}     # total Planck calibration\n")
        path = os.path.join(directory, f"{name}.dataset")
        lines = [
            f"name = {name}",
            "calibration_param = planck_calib.paramnames",
            f"use_cl = {use_cl}",
            f"data = {name}_data.txt",
            f"blmin = {name}_bins_min.txt",
            f"blmax = {name}_bins_max.txt",
            f"weights = {name}_weights.txt",
            f"cov_file = {name}_cov.txt",
        ]
        for k, v in (extra or {}).items():
            lines.append(f"{k} = {v}")
        with open(path, "w") as f:
            f.write("\n".join(lines) + "\n")
        return path


def bin_theory(data: PlikLiteData, dl: np.ndarray) -> np.ndarray:
    """Binned C_b for TT|TE|EE from D_l [10, lmax+1] (CMB.f90:315-325), no calibration."""
    w = data.internal_weights()
    out = []
    for f, nb in zip((FIELD_TT, FIELD_TE, FIELD_EE), NBINCL):
        for b in range(nb):
            lo, hi = PLMIN + data.blmin[b], PLMIN + data.blmax[b]
            out.append(np.dot(dl[f, lo:hi + 1], w[lo - PLMIN:hi - PLMIN + 1]))
    return np.array(out)


def make_plik_lite(seed: int = 12345) -> PlikLiteData:
    blmin, blmax = plik_bins()
    nl = PLMAX - PLMIN + 1
    wfile = np.empty(nl)
    for lo, hi in zip(blmin, blmax):
        wfile[lo:hi + 1] = 1.0 / (hi - lo + 1)
    proto = PlikLiteData(blmin, blmax, wfile, np.zeros(sum(NBINCL)), np.eye(sum(NBINCL)))
    base = base_theory()
    xb = bin_theory(proto, base)
    nb = xb.size
    g = gaussians(seed, nb + nb * nb)
    X = xb * (1.0 + 0.01 * g[:nb])
    A = g[nb:].reshape(nb, nb)
    # sigma_b = 2% of |X_b|, floored at 0.2% of the block rms so that TE bins
    # crossing zero do not make the covariance singular (cond ~1e5, not ~1e13)
    sig = np.empty(nb)
    o = 0
    for n in NBINCL:
        blk = X[o:o + n]
        sig[o:o + n] = 0.02 * np.sqrt(blk ** 2 + (0.1 * np.sqrt(np.mean(blk ** 2))) ** 2)
        o += n
    M = np.eye(nb) + 0.05 * (A @ A.T) / nb
    cov = sig[:, None] * M * sig[None, :]
    cov = 0.5 * (cov + cov.T)
    return PlikLiteData(blmin, blmax, wfile, X, cov)


def _walker_mode_amplitudes(seeds: np.ndarray) -> np.ndarray:
    """Five N(0,1) amplitudes per walker; walker stream = its own seed (vectorised)."""
    with np.errstate(over="ignore"):
        i = np.arange(1, 11, dtype=np.uint64)[None, :]
        z = (seeds.astype(np.uint64)[:, None] + i * _GOLDEN) & _M64
        z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & _M64
        z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & _M64
        z = z ^ (z >> np.uint64(31))
    u = (z >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)
    u1 = 1.0 - u[:, 0::2]
    u2 = u[:, 1::2]
    return np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)


def walker_theory(n_walkers: int, seed: int = 0xC05A0C, lmax: int = PLMAX,
                  first_walker: int = 0, n_fields: int = N_FIELDS,
                  ld_field: int | None = None) -> np.ndarray:
    """Per-walker D_l, shape [W, n_fields, ld_field] (l = 0..lmax, zero padded).

    D_l^w = base_l * (1 + 0.01 s_w(l)),
    s_w(l) = sum_{m=1..5} a_{w,m} cos(pi m (l-2)/(lmax-2)), a ~ N(0,1) from the
    splitmix64 stream ``seed + walker``. Field order is the Theory%Cls(i,j)
    lower-triangle order TT, TE, EE, BT, BE, BB, PT, PE, PB, PP.
    """
    ld = lmax + 1 if ld_field is None else ld_field
    base = base_theory(lmax)[:n_fields]
    ell = np.arange(lmax + 1, dtype=np.float64)
    modes = np.cos(np.pi * np.arange(1, 6)[:, None] * (ell[None, :] - 2.0) / (lmax - 2.0))
    out = np.zeros((n_walkers, n_fields, ld))
    chunk = 256
    for c0 in range(0, n_walkers, chunk):
        c1 = min(n_walkers, c0 + chunk)
        a = _walker_mode_amplitudes(np.arange(seed + first_walker + c0, seed + first_walker + c1))
        s = 1.0 + 0.01 * (a @ modes)
        out[c0:c1, :, :lmax + 1] = base[None, :, :] * s[:, None, :]
    return out


def walker_calibrations(n_walkers: int, seed: int = 0xCA1, first_walker: int = 0) -> np.ndarray:
    g = gaussians(seed, first_walker + n_walkers)[first_walker:]
    return 1.0 + 0.0025 * g


def chain_ensemble(n_chains: int, n_samples: int, n: int, seed: int, spread: float) -> np.ndarray:
    """Samples [n_chains, n_samples, n] of correlated Gaussian 'chains' whose
    centres scatter by ``spread`` (in units of the marginal width): a
    convergence-statistics test input with R-1 of order spread^2."""
    g = gaussians(seed, n * n + n_chains * n + n_chains * n_samples * n)
    A = g[:n * n].reshape(n, n)
    L = np.linalg.cholesky(np.eye(n) + 0.5 * (A @ A.T) / n)
    off = spread * g[n * n:n * n + n_chains * n].reshape(n_chains, n)
    z = g[n * n + n_chains * n:].reshape(n_chains, n_samples, n)
    return (off[:, None, :] + z) @ L.T


# ---------------------------------------------------------------------------
# SPTpol synthetic datasets.  The SPTpol 500d data files are not shipped with
# the reference (no data/ directory or .ini refers to them), so the SPTPOL_TEEE
# and SPTPOL_BB likelihoods are exercised on synthetic data written in the
# exact on-disk formats their readers expect:
#   SPTpol_TEEE_ReadIni / InitSPTpolData  source/CMB_SPTpol_TEEE_2017.f90:56-352
#   SPTpol_BB_ReadIni / InitSPTpolBBData  source/CMB_SPTpol_BB_2019.f90:56-438
# Shapes follow the published analyses (Henning et al. 2018: TE/EE, 56 bins,
# 50 < l < 8000, two beam modes; Sayre et al. 2020: BB 150x150 / 95x150 /
# 95x95, 7 bins, seven beam modes).

def _smooth_windows(lmin: int, lmax: int, edges: list[tuple[int, int]]) -> np.ndarray:
    """Dense window columns [lmax-lmin+1, nbin]: a sin^2-tapered top hat over
    each bin widened by half a bin on both sides, normalised to unit sum."""
    ell = np.arange(lmin, lmax + 1, dtype=np.float64)
    out = np.zeros((ell.size, len(edges)))
    for b, (lo, hi) in enumerate(edges):
        w = hi - lo + 1
        a, z = max(lmin, lo - w // 2), min(lmax, hi + w // 2)
        m = (ell >= a) & (ell <= z)
        x = (ell[m] - a + 0.5) / (z - a + 1.0)
        v = np.sin(np.pi * x) ** 2
        out[m, b] = v / v.sum()
    return out


def _spd_cov(vals: np.ndarray, g: np.ndarray, frac: float) -> np.ndarray:
    n = vals.size
    A = g[:n * n].reshape(n, n)
    sig = frac * np.sqrt(vals ** 2 + (0.1 * np.sqrt(np.mean(vals ** 2))) ** 2)
    M = np.eye(n) + 0.05 * (A @ A.T) / n
    cov = sig[:, None] * M * sig[None, :]
    return 0.5 * (cov + cov.T)


@dataclass
class SptpolTEEEData:
    lmin: int
    lmax: int
    windows: np.ndarray     # [lmax-lmin+1, 2 nbin], TE columns then EE
    spec: np.ndarray        # [3, nbin]  TE, EE, TT
    cov: np.ndarray         # [2 nbin, 2 nbin]
    beam_err: np.ndarray    # [2, 2 nbin]

    PARAMS = ("kappa", "czero_psTE_150", "czero_psEE_150", "ADust_TE", "alphaDust_TE", "ADust_EE",
              "alphaDust_EE", "mapTcal", "mapPcal", "beam1", "beam2")

    @property
    def nbin(self) -> int:
        return self.spec.shape[1]

    def write(self, directory: str, extra: dict | None = None) -> str:
        d = os.path.abspath(directory)
        os.makedirs(os.path.join(d, "sptpol_windows"), exist_ok=True)
        nb, nall = self.nbin, 2 * self.nbin
        with open(os.path.join(d, "sptpol_TEEE.desc"), "w") as f:
            f.write(f"{nb} 1\n{self.lmin} {self.lmax}\n")
        with open(os.path.join(d, "sptpol_TEEE_bp.txt"), "w") as f:
            for i in range(3):
                for j in range(nb):
                    f.write(f"{j + 1} {self.spec[i, j]:.17e}\n")
        # direct-access records of nall doubles, record i = cov(:, i)
        np.ascontiguousarray(self.cov.T, dtype="<f8").tofile(os.path.join(d, "sptpol_TEEE_cov.bin"))
        ell = np.arange(self.lmin, self.lmax + 1)
        for i in range(nall):
            np.savetxt(os.path.join(d, "sptpol_windows", f"window_{i + 1}"),
                       np.column_stack([ell, self.windows[:, i]]), fmt=["%d", "%.17e"])
        with open(os.path.join(d, "sptpol_TEEE_beam.txt"), "w") as f:
            for t in range(self.beam_err.shape[0]):
                for j in range(nall):
                    f.write(f"{j + 1} {self.beam_err[t, j]:.17e}\n")
        with open(os.path.join(d, "sptpol_TEEE.paramnames"), "w") as f:
            for p in self.PARAMS:
                f.write(f"{p}    {p}\n")
        lines = [
            "sptpol_TEEE_params_file = " + os.path.join(d, "sptpol_TEEE.paramnames"),
            "sptpol_TEEE_desc_file = " + os.path.join(d, "sptpol_TEEE.desc"),
            "sptpol_TEEE_bp_file = " + os.path.join(d, "sptpol_TEEE_bp.txt"),
            "sptpol_TEEE_cov_file = " + os.path.join(d, "sptpol_TEEE_cov.bin"),
            "sptpol_TEEE_window_dir = " + os.path.join(d, "sptpol_windows") + "/",
            "sptpol_TEEE_beam_file = " + os.path.join(d, "sptpol_TEEE_beam.txt"),
        ]
        for k, v in (extra or {}).items():
            lines.append(f"{k} = {v}")
        path = os.path.join(d, "sptpol_TEEE.dataset")
        with open(path, "w") as f:
            f.write("\n".join(lines) + "\n")
        return path


def sptpol_teee_edges() -> list[tuple[int, int]]:
    edges = [(51 + 50 * i, 100 + 50 * i) for i in range(50)]
    edges += [(2551, 3000), (3001, 3500), (3501, 4000), (4001, 5000), (5001, 6500), (6501, 7950)]
    return edges


def make_sptpol_teee(seed: int = 2017) -> SptpolTEEEData:
    lmin, lmax = 50, 8000
    edges = sptpol_teee_edges()
    nb = len(edges)
    win1 = _smooth_windows(lmin, lmax, edges)
    base = base_theory(lmax + 1)
    g = gaussians(seed, 3 * nb + 4 * nb * nb + 4 * nb)
    spec = np.zeros((3, nb))
    for k, f in enumerate((FIELD_TE, FIELD_EE, FIELD_TT)):
        spec[k] = (win1.T @ base[f, lmin:lmax + 1]) * (1.0 + 0.02 * g[k * nb:(k + 1) * nb])
    cov = _spd_cov(spec[:2].ravel(), g[3 * nb:], 0.03)
    beam = 0.01 * g[3 * nb + 4 * nb * nb:].reshape(2, 2 * nb)
    return SptpolTEEEData(lmin, lmax, np.hstack([win1, win1]), spec, cov, beam)


@dataclass
class SptpolBBData:
    lmin: int
    lmax: int
    eff_freqs: tuple        # eff dust frequencies (150 band first, decreasing)
    edges: list
    windows: np.ndarray     # [lmax-lmin+1, 3 nbin]: 150x150, 95x150, 95x95
    spec: np.ndarray        # [3, nbin] same order
    cov: np.ndarray         # [3 nbin, 3 nbin]
    beam_err: np.ndarray    # [7, 3 nbin]
    r_template: np.ndarray  # [lmax_t + 1] BB D_l of r = 1 tensors (l = 0..)

    PARAMS = ("Abb", "r_sptpol", "const_bb", "Add_150", "Pois_150", "Pois_95x150", "Pois_95",
              "MapBcal150", "MapBcal95") + tuple(f"bbbeam{i}" for i in range(1, 8))

    @property
    def nbin(self) -> int:
        return self.spec.shape[1]

    def write(self, directory: str, extra: dict | None = None, with_r_template: bool = True) -> str:
        d = os.path.abspath(directory)
        os.makedirs(d, exist_ok=True)
        nb, nall = self.nbin, 3 * self.nbin
        with open(os.path.join(d, "sptpol_BB.desc"), "w") as f:
            f.write(f"{nb} 2\n{self.lmin} {self.lmax}\n{self.eff_freqs[0]!r}\n{self.eff_freqs[1]!r}\n")
        with open(os.path.join(d, "sptpol_BB_bp.txt"), "w") as f:
            f.write("# lcenter lmin lmax BB_95x95 BB_95x150 BB_150x150\n")
            for b, (lo, hi) in enumerate(self.edges):
                f.write(f"{(lo + hi) / 2:.1f} {lo} {hi} {self.spec[2, b]:.17e} {self.spec[1, b]:.17e} "
                        f"{self.spec[0, b]:.17e}\n")
        np.ascontiguousarray(self.cov.T, dtype="<f8").tofile(os.path.join(d, "sptpol_BB_cov.bin"))
        with open(os.path.join(d, "sptpol_BB_windows.bin"), "wb") as f:
            f.write(np.array([self.lmin, self.lmax], dtype="<i4").tobytes())
            f.write(np.asfortranarray(self.windows, dtype="<f8").tobytes(order="F"))
        with open(os.path.join(d, "sptpol_BB_beam.bin"), "wb") as f:
            f.write(np.array([nall, self.beam_err.shape[0]], dtype="<i4").tobytes())
            f.write(np.ascontiguousarray(self.beam_err, dtype="<f8").tobytes())
        with open(os.path.join(d, "sptpol_BB.paramnames"), "w") as f:
            for p in self.PARAMS:
                f.write(f"{p}    {p}\n")
        lines = [
            "sptpol_BB_params_file = " + os.path.join(d, "sptpol_BB.paramnames"),
            "sptpol_BB_desc_file = " + os.path.join(d, "sptpol_BB.desc"),
            "sptpol_BB_bp_file = " + os.path.join(d, "sptpol_BB_bp.txt"),
            "sptpol_BB_cov_file = " + os.path.join(d, "sptpol_BB_cov.bin"),
            "sptpol_BB_window_file = " + os.path.join(d, "sptpol_BB_windows.bin"),
            "sptpol_BB_beam_file = " + os.path.join(d, "sptpol_BB_beam.bin"),
        ]
        if with_r_template:
            tp = os.path.join(d, "r_template_totcls.dat")
            with open(tp, "w") as f:
                f.write("#    L    TT             EE             BB             TE\n")
                for l in range(2, self.r_template.size):
                    t = self.r_template[l]
                    f.write(f"{l:5d} {40 * t:.8e} {0.5 * t:.8e} {t:.8e} {3 * t:.8e}\n")
            lines.append("r_template_file = " + tp)
        with open(os.path.join(d, "sptpol_blind_abb.bin"), "wb") as f:
            f.write(np.array([0.0125], dtype="<f8").tobytes())
        for k, v in (extra or {}).items():
            lines.append(f"{k} = {v}")
        path = os.path.join(d, "sptpol_BB.dataset")
        with open(path, "w") as f:
            f.write("\n".join(lines) + "\n")
        return path


def make_sptpol_bb(seed: int = 2019) -> SptpolBBData:
    lmin, lmax = 50, 2350
    edges = [(51, 250), (251, 500), (501, 750), (751, 1000), (1001, 1350), (1351, 1800), (1801, 2300)]
    nb = len(edges)
    win1 = _smooth_windows(lmin, lmax, edges)
    base = base_theory(lmax + 1)
    g = gaussians(seed, 3 * nb + 9 * nb * nb + 21 * nb)
    spec = np.zeros((3, nb))
    fg = (0.06, 0.12, 0.25)                  # rough foreground excess per band
    for k in range(3):
        spec[k] = (win1.T @ base[FIELD_BB, lmin:lmax + 1]) * (1.0 + fg[k]) * (1.0 + 0.05 * g[k * nb:(k + 1) * nb])
    cov = _spd_cov(spec.ravel(), g[3 * nb:], 0.08)
    beam = 0.005 * g[3 * nb + 9 * nb * nb:].reshape(7, 3 * nb)
    lt = 3000
    ell = np.arange(lt + 1, dtype=np.float64)
    rt = np.zeros(lt + 1)
    rt[2:] = 0.06 * (ell[2:] / 80.0) ** 1.0 * np.exp(-(ell[2:] / 120.0) ** 1.5)
    return SptpolBBData(lmin, lmax, (152.3, 96.2), edges, np.hstack([win1, win1, win1]), spec, cov, beam, rt)


# ---------------------------------------------------------------------------
# BK15 (BASELINE configs[4]): the reference ships data/BK15 without its
# bandpower covariance (BK15_dust.dataset: covmat_fiducial = BK15_covmat_dust.dat
# is absent), so a synthetic SPD covariance of the file's shape is written next
# to the real files: (300 spectra x 9 bins)^2, text, bin-major as ReadCovmat
# expects (CMBlikes.f90:785-795).  The 78 B x B spectra (the BK15.ini B-only
# selection) carry a dense correlated block across all bins; every other
# spectrum is diagonal, so any map selection stays positive definite.

def _bk15_order(dataset_path: str) -> list[str]:
    with open(dataset_path) as f:
        for line in f:
            s = line.strip()
            if s.startswith("covmat_cl"):
                return s.split("=", 1)[1].split()
    raise ValueError("covmat_cl missing in " + dataset_path)


def write_refdata_extras(d: str) -> None:
    """Files the tests add beside the reference's extracted data (``d``): the
    synthetic BK15 covariance (configs[4]) and a one-name calibration parameter
    file for BKPLANCK + calibration_param."""
    if os.path.isdir(os.path.join(d, "BK15")):
        write_bk15_covmat(os.path.join(d, "BK15"))
    if os.path.isdir(os.path.join(d, "BKPlanck")):
        with open(os.path.join(d, "BKPlanck", "bk_cal.paramnames"), "w") as f:
            f.write("calBK   c_{BK}\n")


def write_bk15_covmat(bk15_dir: str, seed: int = 1515, rank: int = 24) -> str:
    """Write BK15_covmat_dust.dat into ``bk15_dir`` (the extracted data/BK15)."""
    order = _bk15_order(os.path.join(bk15_dir, "BK15_dust.dataset"))
    ncl, nbin = len(order), 9
    fid = np.loadtxt(os.path.join(bk15_dir, "BK15_fiducial_dust.dat"), ndmin=2)[:nbin, 1:ncl + 1]
    noi = np.loadtxt(os.path.join(bk15_dir, "BK15_noise.dat"), ndmin=2)[:nbin, 1:ncl + 1]
    # sigma of spectrum A x B ~ 0.15 sqrt((C_AA + N_AA)(C_BB + N_BB)) (Knox-like scaling)
    auto = {c.split("x")[0]: i for i, c in enumerate(order) if c.split("x")[0] == c.split("x")[1]}
    tot = np.abs(fid) + np.abs(noi)
    scale = np.empty_like(tot)                                 # [bin][cl]
    for i, c in enumerate(order):
        a, b = c.split("x")
        scale[:, i] = 0.15 * np.sqrt(tot[:, auto[a]] * tot[:, auto[b]]) + 1e-4
    n = ncl * nbin
    sig = scale.ravel()                                        # index (bin - 1) * ncl + cl
    bb = [i for i, c in enumerate(order) if c.count("_B") == 2]
    dense = np.array([b * ncl + c for b in range(nbin) for c in bb])
    m = dense.size
    g = gaussians(seed, m * rank)
    B = g.reshape(m, rank)
    corr = np.eye(m) + 0.3 * (B @ B.T) / rank
    d = 1.0 / np.sqrt(np.diag(corr))
    corr = corr * d[:, None] * d[None, :]
    in_dense = np.full(n, -1)
    in_dense[dense] = np.arange(m)
    path = os.path.join(bk15_dir, "BK15_covmat_dust.dat")
    with open(path, "w") as f:
        for i in range(n):
            row = ["0"] * n
            if in_dense[i] >= 0:
                vals = corr[in_dense[i]] * sig[i] * sig[dense]
                for jj, j in enumerate(dense):
                    row[j] = repr(float(vals[jj]))
            else:
                row[i] = repr(float(sig[i] * sig[i]))
            f.write(" ".join(row))
            f.write("\n")
    return path


# ------------------------------------------------------------------ unbinned exact
# CMBlikes like_approx = exact (ExactChiSq, CMBlikes.f90:967-979) needs an
# unbinned dataset: per-l observed spectra cl_hat and noise cl_noise.  No such
# dataset ships with the reference, so this writes one in the CMBLike2 format
# ReadClArr reads (:146-193): Chat_l is a Wishart draw with round((2l+1) fksy)
# degrees of freedom around theory + noise (a full-sky estimator's scatter).
EXACT_PAIRS = ("TT", "TE", "EE", "TB", "EB", "BB")     # i >= j over T E B (ElementsToMatrix order)
_EXACT_FIELD = {"TT": FIELD_TT, "TE": FIELD_TE, "EE": FIELD_EE, "TB": FIELD_BT, "EB": FIELD_BE, "BB": FIELD_BB}


@dataclass
class ExactData:
    lmin: int
    lmax: int
    clhat: np.ndarray       # [lmax+1, 6] (EXACT_PAIRS columns), zero below lmin
    noise: np.ndarray       # [lmax+1, 6]

    def write(self, directory: str, fields: str = "T E B", extra: dict | None = None,
              hat_includes_noise: bool = False) -> str:
        d = os.path.abspath(directory)
        os.makedirs(d, exist_ok=True)
        hdr = "#    L " + " ".join(f"{p:>24s}" for p in EXACT_PAIRS)
        ell = np.arange(self.lmin, self.lmax + 1)
        hat = self.clhat + (self.noise if hat_includes_noise else 0.0)
        for fn, arr in (("exact_clhat.dat", hat), ("exact_noise.dat", self.noise)):
            with open(os.path.join(d, fn), "w") as f:
                f.write(hdr + "\n")
                for l in ell:
                    f.write(f"{l:6d} " + " ".join(f"{v:24.17e}" for v in arr[l]) + "\n")
        with open(os.path.join(d, "exact_cal.paramnames"), "w") as f:
            f.write("calPlanck    y_{\\rm cal}\n")
        lines = ["dataset_format = CMBLike2", "like_approx = exact", f"fields_use = {fields}",
                 f"cl_lmin = {self.lmin}", f"cl_lmax = {self.lmax}", "binned = F",
                 "cl_hat_file = exact_clhat.dat", "cl_noise_file = exact_noise.dat",
                 f"cl_hat_includes_noise = {'T' if hat_includes_noise else 'F'}"]
        for k, v in (extra or {}).items():
            lines.append(f"{k} = {v}")
        path = os.path.join(d, "exact.dataset")
        with open(path, "w") as f:
            f.write("\n".join(lines) + "\n")
        return path


def make_exact(lmin: int = 2, lmax: int = 400, fksy: float = 1.0, seed: int = 1979) -> ExactData:
    base = base_theory(max(lmax, 2))
    ell = np.arange(lmax + 1, dtype=np.float64)
    white = ell * (ell + 1) / (2 * np.pi)
    noise = np.zeros((lmax + 1, 6))
    noise[:, 0] = 1e-4 * white                  # TT
    noise[:, 2] = 2e-4 * white                  # EE
    noise[:, 5] = 2e-4 * white                  # BB
    clhat = np.zeros((lmax + 1, 6))
    for l in range(lmin, lmax + 1):
        C = np.zeros((3, 3))
        for k, p in enumerate(EXACT_PAIRS):
            i, j = "TEB".index(p[0]), "TEB".index(p[1])
            C[i, j] = C[j, i] = base[_EXACT_FIELD[p], l] + noise[l, k]
        nu = max(3, int(round((2 * l + 1) * fksy)))
        x = np.linalg.cholesky(C) @ gaussians(seed + l, 3 * nu).reshape(3, nu)
        S = x @ x.T / nu
        for k, p in enumerate(EXACT_PAIRS):
            i, j = "TEB".index(p[0]), "TEB".index(p[1])
            clhat[l, k] = S[i, j] - noise[l, k]
    return ExactData(lmin, lmax, clhat, noise)


# SMICA (TSmica_planck, source/CMBlikes.f90:1262-1339): no SMICA dataset ships
# with the reference, so a synthetic binned TT CMBLike2 dataset in its format
# (CMBLikes_ReadIni :466-749) with the SMICA nuisance_params file: the five
# foreground parameters, a calibration, and the derived D_l(2000).
SMICA_PARAMS = (("A1_smica", "A_1"), ("n1_smica", "n_1"), ("n1run_smica", "n_{1,\\rm run}"),
                ("A2_smica", "A_2"), ("n2_smica", "n_2"), ("cal_smica", "y_{\\rm cal}"))
SMICA_FG = (30.0, 1.2, 0.0, 20.0, 0.5)     # fiducial A1 n1 n1run A2 n2 (D_l muK^2 at l = 2000)


def smica_edges() -> list[tuple[int, int]]:
    return [(30 + 45 * i, 74 + 45 * i) for i in range(54)]      # 54 bins, l 30..2459


@dataclass
class SmicaData:
    lmin: int
    lmax: int
    windows: np.ndarray     # [lmax-lmin+1, nbin]
    clhat: np.ndarray       # [nbin] binned TT (signal)
    clfid: np.ndarray       # [nbin] fiducial (HL)
    noise: np.ndarray       # [nbin] noise (HL)
    cov: np.ndarray         # [nbin, nbin]

    def write(self, directory: str, like_approx: str = "gaussian", extra: dict | None = None) -> str:
        d = os.path.abspath(directory)
        os.makedirs(os.path.join(d, "smica_windows"), exist_ok=True)
        nb = self.clhat.size
        ell = np.arange(self.lmin, self.lmax + 1)
        for b in range(nb):
            np.savetxt(os.path.join(d, "smica_windows", f"window{b + 1}.dat"),
                       np.column_stack([ell, self.windows[:, b]]), fmt=["%d", "%.17e"])
        for fn, v in (("smica_clhat.dat", self.clhat), ("smica_clfid.dat", self.clfid),
                      ("smica_noise.dat", self.noise)):
            with open(os.path.join(d, fn), "w") as f:
                f.write("#    L    TT\n")
                for b in range(nb):
                    f.write(f"{b + 1:6d} {v[b]:24.17e}\n")
        np.savetxt(os.path.join(d, "smica_cov.dat"), self.cov, fmt="%.17e")
        with open(os.path.join(d, "smica.paramnames"), "w") as f:
            for n, lab in SMICA_PARAMS:
                f.write(f"{n}    {lab}\n")
            f.write("Dl2000_smica*    D_{2000}\n")
        with open(os.path.join(d, "smica_cal.paramnames"), "w") as f:
            f.write("calPlanck    y_{\\rm cal}\n")
        lines = ["dataset_format = CMBLike2", f"like_approx = {like_approx}", "fields_use = T", "binned = T",
                 f"nbins = {nb}", f"cl_lmin = {self.lmin}", f"cl_lmax = {self.lmax}",
                 "bin_window_files = smica_windows/window%u.dat", "bin_window_in_order = TT",
                 "cl_hat_file = smica_clhat.dat", "covmat_cl = TT", "covmat_fiducial = smica_cov.dat",
                 "nuisance_params = smica.paramnames"]
        if like_approx == "HL":
            lines += ["cl_fiducial_file = smica_clfid.dat", "cl_noise_file = smica_noise.dat"]
        for k, v in (extra or {}).items():
            lines.append(f"{k} = {v}")
        path = os.path.join(d, "smica.dataset")
        with open(path, "w") as f:
            f.write("\n".join(lines) + "\n")
        return path


def smica_foreground(ells: np.ndarray, P) -> np.ndarray:
    """The SMICA TT foreground (CMBlikes.f90:1314-1317) in numpy, for data making."""
    A1, n1, n1run, A2, n2 = P[:5]
    r = np.log(ells / 2000.0)
    return A1 * np.exp(n1 * r + n1run / 2 * r ** 2) + A2 * (ells / 2000.0) ** n2


def make_smica(seed: int = 2015) -> SmicaData:
    lmin, lmax = 2, 2508
    edges = smica_edges()
    nb = len(edges)
    win = _smooth_windows(lmin, lmax, edges)
    base = base_theory(lmax)
    ells = np.arange(lmin, lmax + 1, dtype=np.float64)
    tt = base[FIELD_TT, lmin:lmax + 1] + smica_foreground(ells, SMICA_FG)
    g = gaussians(seed, nb + nb * nb + nb)
    binned = win.T @ tt
    clhat = binned * (1.0 + 0.01 * g[:nb])
    noise = 0.02 * binned * (1.0 + 0.1 * np.abs(g[nb + nb * nb:]))
    cov = _spd_cov(binned, g[nb:nb + nb * nb], 0.015)
    return SmicaData(lmin, lmax, win, clhat, binned, noise, cov)


def _py_gaussians(seed: int, n: int) -> list[float]:
    """gaussians() restated on Python floats and libm (math): the splitmix64
    uniforms are exact, and every later operation is one correctly ordered
    IEEE step, so two hosts of this image produce the same bits (numpy's
    vectorised log/cos may pick a different SIMD path per CPU)."""
    import math
    u = uniforms(seed, 2 * n).tolist()
    return [math.sqrt(-2.0 * math.log(1.0 - u[2 * i])) * math.cos(2.0 * math.pi * u[2 * i + 1]) for i in range(n)]


def chain_problem(n: int, seed: int, extra: dict | None = None):
    """The test_likelihood Gaussian of a sampler golden chain
    (oracle/gen_golden.py CHAIN_CASES): SPD covariance over n used
    parameters, centre, bounds, priors, start point, plus extra["fixed"] fixed
    parameters (appended, bounds pinned at their value, each with a Gaussian
    prior) and extra["lincomb"] linear-combination priors over all
    parameters.  Pure-Python arithmetic in a fixed order (see _py_gaussians),
    so the GPU box rebuilds exactly the problem the reference ran on.

    Returns (cov, center, pmin, pmax, pmean, pstd, P0, lincombs)."""
    import math
    extra = extra or {}
    g = _py_gaussians(seed, n * n + 3 * n)
    A = [g[i * n:(i + 1) * n] for i in range(n)]
    sig = [0.5 + abs(x) for x in g[n * n:n * n + n]]
    corr = [[0.0] * n for _ in range(n)]
    for i in range(n):
        for j in range(n):
            s = 0.0
            for k in range(n):
                s += A[i][k] * A[j][k]
            corr[i][j] = (1.0 if i == j else 0.0) + 0.3 * s / n
    d = [1.0 / math.sqrt(corr[i][i]) for i in range(n)]
    cov = np.array([[corr[i][j] * d[i] * d[j] * sig[i] * sig[j] for j in range(n)] for i in range(n)])
    center = [g[n * n + n + i] for i in range(n)]
    pmin = [center[i] - 4.0 * sig[i] for i in range(n)]
    pmax = [center[i] + 4.0 * sig[i] for i in range(n)]
    pmean = [0.0] * n
    pstd = [0.0] * n
    pmean[-1] = center[-1] + 0.2 * sig[-1]
    pstd[-1] = 2.0 * sig[-1]
    P0 = [center[i] + 0.5 * sig[i] * g[n * n + 2 * n + i] for i in range(n)]
    nf = extra.get("fixed", 0)
    fv = [0.3 + 0.1 * k for k in range(nf)]
    center += fv
    pmin += fv
    pmax += fv
    pmean += [v + 0.05 for v in fv]
    pstd += [0.1] * nf
    P0 += fv
    lin = []
    gl = _py_gaussians(seed + 99, 3 * max(1, extra.get("lincomb", 0)))
    for k in range(extra.get("lincomb", 0)):
        w = [0.0] * (n + nf)
        i, j = (2 * k) % n, (2 * k + 5) % n
        w[i], w[j] = 1.0, 0.5 + 0.1 * gl[3 * k]            # e.g. SZComb = A_kSZ + 1.6 A_tSZ
        if nf:
            w[n] = 0.25                                      # fixed parameters enter dot_product(Comb, P)
        s = 0.0
        for a, b in zip(w, center):
            s += a * b
        lin.append({"weights": w, "mean": s + 0.3 * gl[3 * k + 1], "std": 1.5 + abs(gl[3 * k + 2])})
    arr = [np.array(v, dtype=np.float64) for v in (center, pmin, pmax, pmean, pstd, P0)]
    return (cov, *arr, lin)
