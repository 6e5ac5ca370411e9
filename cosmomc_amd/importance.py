"""Importance sampling (CosmoMC ``action = 1``) with batched GPU re-evaluation.

Mirrors TImportanceSampler (reference source/ImportanceSampling.f90):

* ``ReadParams`` keys (:55-88): redo_likelihoods, redo_theory, redo_outroot,
  redo_likeoffset, redo_temp, redo_change_like_only, redo_nochange,
  redo_skip, redo_thin, redo_auto_likescale, redo_max_logLike_diff,
  redo_auto_likescale_count;
* ``ImportanceSample`` (:105-411) on text chains (the ``redo_from_text``
  path, :142-160 / :240-245): every row ``mult like P(params_used)`` gets
  ``truelike = GetLogLikePost`` (calclike.f90:334-354: bounds -> logZero,
  data likelihoods, Gaussian priors, each divided by the temperature),
  ``weight = exp(like - truelike + redo_likeoffset)`` (0 for logZero) and
  ``mult *= weight`` unless redo_change_like_only / redo_nochange; rows with
  mult > 1e-100 are written (:365-377); the automatic offset restart
  (:340-363) and the summary statistics (:395-406) follow the reference.

The rows are evaluated ``W`` at a time on the GPU (GPUEvaluator): a
BatchedMCMC with the new likelihoods registered evaluates GetLogLike at the
rows (``cmbs_set_start``) after ``theory_fn`` filled each likelihood's theory
buffer for the batch (``redo_theory``; GetTheoryForImportance, the CAMB call of
the reference, is the caller's).  Without redo_theory every row is scored on
the cached theory the buffers hold.

Out of scope: the binary ``.data`` path (redo_add / redo_like_name need the
per-likelihood values stored there), ``NonBaseParameterPriors`` of a
cosmology parameterization (no CAMB here), redo_output_txt_theory.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field

import numpy as np

from .chains import fortran_e

LOGZERO = 1e30


@dataclass
class ImportanceSettings:
    redo_likelihoods: bool = False
    redo_theory: bool = False
    redo_outroot: str = ""
    redo_likeoffset: float = 0.0
    redo_temp: float = 1.0
    redo_change_like_only: bool = False
    redo_nochange: bool = False
    redo_skip: float = 100
    redo_thin: int = 1
    redo_auto_likescale: bool = True
    redo_max_logLike_diff: float = 10.0
    redo_auto_likescale_count: int = 5

    @classmethod
    def from_ini(cls, ini) -> "ImportanceSettings":
        """TImportanceSampler_ReadParams (ImportanceSampling.f90:55-88); ``ini``
        maps key -> string (e.g. cosmomc_amd.ini.IniFile)."""
        s = cls()

        def get(k):
            try:
                v = ini[k]
            except KeyError:
                return None
            return None if v in (None, "") else str(v)

        def logical(v):
            return v.strip().upper().lstrip(".").startswith("T")

        def num(v):
            return float(v.replace("d", "e").replace("D", "e"))
        for k in ("redo_likelihoods", "redo_theory", "redo_change_like_only", "redo_nochange",
                  "redo_auto_likescale"):
            v = get(k)
            if v is not None:
                setattr(s, k, logical(v))
        for k in ("redo_likeoffset", "redo_skip", "redo_max_logLike_diff", "redo_temp"):
            v = get(k)
            if v is not None:
                setattr(s, k, num(v))
        for k in ("redo_thin", "redo_auto_likescale_count"):
            v = get(k)
            if v is not None:
                setattr(s, k, int(v))
        v = get("redo_outroot")
        if v is not None:
            s.redo_outroot = v
        for k in ("redo_add", "redo_like_name"):
            v = get(k)
            if v is not None and (k == "redo_like_name" or logical(v)):
                raise ValueError("redo_add and/or redo_like_name require .data files, not from text")
        if s.redo_thin < 1:
            raise ValueError("redo_thin: value < min")
        return s


@dataclass
class ImportanceResult:
    num_used: int = 0
    weight_min: float = 1e30
    weight_max: float = -1e30
    mult_sum: float = 0.0
    mult_ratio: float = 0.0
    mult_max: float = -1e30
    max_like: float = LOGZERO
    max_truelike: float = LOGZERO
    likeoffset: float = 0.0
    rows: list = field(default_factory=list)       # (mult, truelike, P_used) written

    @property
    def mean_mult(self):
        return self.mult_sum / self.num_used if self.num_used else 0.0

    @property
    def mean_weight(self):                          # approx evidence ratio (:399)
        return self.mult_ratio / self.num_used if self.num_used else 0.0

    @property
    def effective_samples(self):                    # :400
        return self.mult_sum / self.mult_max if self.mult_max > 0 else 0.0


def read_chain_rows(path: str) -> np.ndarray:
    """IO_ReadChainRow (IO.f90): whitespace rows ``mult like P...``."""
    rows = []
    with open(path) as f:
        for line in f:
            s = line.strip()
            if s and not s.startswith("#"):
                rows.append([float(x.replace("D", "E").replace("d", "e")) for x in s.split()])
    n = len(rows[0]) if rows else 0
    return np.array(rows, dtype=np.float64).reshape(len(rows), n)


class GPUEvaluator:
    """GetLogLikePost for batches of parameter rows on the GPU.

    sampler: a BatchedMCMC (W walkers, temperature = redo_temp, bounds and
    priors of the new run) with the new likelihoods registered;
    theory_fn(P [W, num_params] numpy) fills the registered theory buffers
    for the rows (None: every row is scored on the cached theory)."""

    def __init__(self, sampler, theory_fn=None):
        self.s = sampler
        self.theory_fn = theory_fn
        self.W = sampler.W

    def prior_cut(self, P: np.ndarray) -> np.ndarray:
        """True for rows outside the new run's hard bounds: CheckPriorCuts
        (calclike.f90:320-331) = GetLogLikeBounds (:97-109); the cosmology
        parameterization's NonBaseParameterPriors term is out of scope."""
        return np.any((P > self.s.pmax[None, :]) | (P < self.s.pmin[None, :]), axis=1)

    def __call__(self, P: np.ndarray) -> np.ndarray:
        n = P.shape[0]
        out = np.empty(n)
        for b0 in range(0, n, self.W):
            blk = P[b0:b0 + self.W]
            m = blk.shape[0]
            if m < self.W:                           # pad the last batch with its last row
                blk = np.concatenate([blk, np.repeat(blk[-1:], self.W - m, axis=0)])
            if self.theory_fn is not None:
                self.theory_fn(blk)
            self.s.set_start(blk)                    # GetLogLike at the rows (synchronises)
            _, like, _, _ = self.s.state()
            out[b0:b0 + m] = like[:m]
        return out


def nint(x: float) -> int:
    """Fortran NINT: round half away from zero (Python's round is half-to-even)."""
    return int(math.copysign(math.floor(abs(x) + 0.5), x))


class ImportanceSampler:
    """TImportanceSampler on text chains.

    params_used: 1-based indices into P of the chain columns after mult/like
    (the order the input chain was written in); center: P of the parameters
    the chain does not hold (BaseParams%center, :242); evaluate(P [n,
    num_params]) -> GetLogLikePost of every row (a GPUEvaluator)."""

    def __init__(self, settings: ImportanceSettings, params_used, center, evaluate):
        self.s = settings
        self.params_used = list(params_used)
        self.center = np.asarray(center, dtype=np.float64)
        self.evaluate = evaluate

    def read(self, path):
        """Rows after redo_skip and redo_thin: mult, like, P [n, num_params]."""
        data = read_chain_rows(path)
        skip = self.s.redo_skip
        if skip < 1:                                   # a fraction of the lines (:146-148)
            skip = nint(data.shape[0] * skip)
        num = np.arange(1, data.shape[0] + 1)
        keep = ~((skip >= 1) & (num <= skip))          # num <= redo_skip: cycle (:245)
        data = data[keep]
        mult, like = data[:, 0].copy(), data[:, 1].copy()
        P = np.tile(self.center, (data.shape[0], 1))
        for c, i in enumerate(self.params_used):
            P[:, i - 1] = data[:, 2 + c]
        if self.s.redo_thin > 1:                       # :279-289
            if np.any(np.abs(np.rint(mult) - mult) > 1e-4):
                raise ValueError("redo_thin can only be used with chains with integer weights")
            acc, sel, newm = 0, [], []
            for k, m in enumerate(mult):
                acc += nint(m)
                if acc >= self.s.redo_thin:
                    newm.append(acc // self.s.redo_thin)
                    acc = acc % self.s.redo_thin
                    sel.append(k)
            sel = np.array(sel, dtype=int)
            mult, like, P = np.array(newm, dtype=np.float64), like[sel], P[sel]
        return mult, like, P

    def run(self, in_path: str, out_root: str | None = None) -> ImportanceResult:
        """Importance-sample the chain file ``in_path``; writes out_root.txt
        (GetDist rows through the reference's ChainOutFile format, E16.7,
        settings.f90:109 / ImportanceSampling.f90:221) when out_root is given."""
        mult0, like, P = self.read(in_path)
        cut = getattr(self.evaluate, "prior_cut", None)
        if self.s.redo_likelihoods and cut is not None:
            # rows outside the new prior bounds are skipped before anything is
            # counted (ImportanceSampling.f90:296-302)
            keep = ~cut(P)
            mult0, like, P = mult0[keep], like[keep], P[keep]
        truelike_all = self.evaluate(P) if self.s.redo_likelihoods else like.copy()
        offset = self.s.redo_likeoffset
        redo_loop = 1
        while True:
            r = ImportanceResult(likeoffset=offset)
            restart = False
            for k in range(mult0.size):
                mult = mult0[k]
                if self.s.redo_likelihoods:
                    truelike = truelike_all[k]
                    weight = 0.0 if truelike == LOGZERO else math.exp(like[k] - truelike + offset)
                    if not self.s.redo_change_like_only and not self.s.redo_nochange:
                        mult = mult * weight
                else:
                    truelike, weight = like[k], 1.0
                if self.s.redo_nochange:
                    truelike = like[k]
                r.max_like = min(r.max_like, like[k])
                r.max_truelike = min(r.max_truelike, truelike)
                r.num_used += 1
                r.mult_ratio += weight
                r.mult_sum += mult
                if (self.s.redo_auto_likescale and redo_loop == 1 and r.num_used == self.s.redo_auto_likescale_count
                        and not self.s.redo_change_like_only and not self.s.redo_nochange):
                    diff = r.max_truelike - r.max_like if r.max_truelike != LOGZERO else LOGZERO
                    if abs(diff) > self.s.redo_max_logLike_diff:   # restart with this offset (:357-362)
                        offset = diff
                        redo_loop = 2
                        restart = True
                        break
                if mult > 1e-100:
                    r.rows.append((mult, truelike, P[k, [i - 1 for i in self.params_used]].copy()))
                r.weight_max = max(weight, r.weight_max)
                r.weight_min = min(weight, r.weight_min)
                r.mult_max = max(r.mult_max, mult)
            if not restart:
                break
        if out_root:
            d = os.path.dirname(out_root)
            if d:
                os.makedirs(d, exist_ok=True)
            with open(out_root + ".txt", "w") as f:
                for mult, tl, pu in r.rows:
                    f.write("".join(fortran_e(v, 16) for v in [mult, tl, *pu]) + "\n")
        return r
