"""CosmoMC / GetDist chain files from the batched sampler.

Reference: every accepted move writes the previous point with its
multiplicity, ``mult like values`` (IO_OutputChainRow, source/IO.f90:85-93,
via TChainSampler_MoveDone -> AddNewWeightedPoint, source/MCMC.f90:166-190),
in ChainOutFile's ``'(*(E16.7))'`` (source/settings.f90:109), one ``root_N.txt`` per
chain, plus ``root.paramnames`` and ``root.ranges``.

Here every walker is a chain: the sampler's history ring holds each walker's
current point and -lnL after every step (``cmbs_history_host``); a run of
identical consecutive points is one stay, its length the multiplicity ``mult``
that MoveDone passes on when the chain moves off it.  A run still open at the
end of a block stays pending until the chain leaves the point; like the
reference, the point a chain sits at when the run ends is never written.

MoveDone / AddNewWeightedPoint semantics (MCMC.f90:166-190,
SampleCollector.f90:82-111):
  * ``burn_in`` (MCMC.f90:39, default 2, ini ``burn_in``): a stay is written
    only if num_accept > burn_in when the chain leaves it -- the first
    burn_in + 1 stays are dropped;
  * ``thin`` (the thin_fac MoveDone passes: oversample_fast for
    TMetropolisSampler_GetNewSample :290, 1 for FastParameterSample and the
    dragging sampler :327, :440): acc += mult; when acc >= thin (or thin = 1)
    the row is written with weight acc/thin and acc = mod(acc, thin);
  * stays at logZero are not written; MaxLike / MaxLikeParams track the best
    point a chain has moved off (:182-185).

With ``likelihoods`` given, rows carry the reference's likelihood-derived
columns (AddOutputLikelihoodParams / addLikelihoodDerivedParams,
source/GeneralTypes.f90:671-776): ``chi2_<tag>`` = 2 x each likelihood's -lnL
at the point (``cmbs_history_terms_host``), ``chi2_prior`` = 2 x (like -
sum of terms), and ``chi2_<type>`` sums for every likelihood type used more
than once; ``root.likelihoods`` lists them (OutputDescription, :792-812).
With ``derived`` given, the likelihoods' own derived parameters (the '*'
names of their nuisance .paramnames, e.g. SMICA's D_l(2000)) come first among
the derived columns, as in addLikelihoodDerivedParams (:772-777):
``LikelihoodDerived`` evaluates them on the device for every history row.
"""
from __future__ import annotations

import math
import os

import numpy as np

LOGZERO = 1e30            # settings.f90:114


def fortran_e(x: float, w: int = 17, d: int = 7) -> str:
    """Fortran Ew.d edit descriptor (e.g. E17.7: '   0.1234567E+01')."""
    if x == 0.0 or not math.isfinite(x):
        body = f"0.{'0' * d}E+00" if x == 0.0 else str(x)
        return body.rjust(w)
    e = math.floor(math.log10(abs(x))) + 1
    m = abs(x) / 10.0 ** e
    digits = round(m * 10 ** d)
    if digits >= 10 ** d:                         # rounding carried into the next decade
        digits //= 10
        e += 1
    if digits < 10 ** (d - 1):                    # log10 rounding below the decade
        digits = round(abs(x) / 10.0 ** (e - 1) * 10 ** d)
        e -= 1
    s = f"{'-' if x < 0 else ''}0.{digits:0{d}d}E{'+' if e >= 0 else '-'}{abs(e):02d}"
    return s.rjust(w)


class ChainWriter:
    """Chain files for walkers ``walkers`` (default all) of a BatchedMCMC.

    names / labels / ranges are for the used parameters (params_used order);
    ranges: list of (min, max) or None."""

    def __init__(self, root: str, names, labels=None, ranges=None, walkers=None, first_chain: int = 1,
                 likelihoods=None, burn_in: int = 2, thin: int = 1, derived=None):
        """likelihoods: one (tag, type, name, version) per sampler likelihood,
        in add_likelihood order, to add the chi2_* columns.  burn_in / thin as
        TChainSampler%burn_in and MoveDone's thin_fac (module docstring).
        derived: a LikelihoodDerived (its names, and the columns it computes
        from the history's points)."""
        self.root = root
        self.names = list(names)
        self.labels = list(labels) if labels is not None else list(names)
        self.ranges = ranges
        self.walkers = walkers
        self.first_chain = first_chain
        self.likelihoods = [tuple(x) for x in likelihoods] if likelihoods else []
        self.like_derived = derived
        self.pending = {}                          # walker -> [point values (like, P..., chi2...), count]
        self.next_step = None
        self.burn_in, self.thin = int(burn_in), max(1, int(thin))
        self.num_accept = {}                       # walker -> stays left so far (MoveDone's num_accept)
        self.acc = {}                              # walker -> AddNewWeightedPoint acc
        self.max_like = {}                         # walker -> (MaxLike, point values)
        d = os.path.dirname(root)
        if d:
            os.makedirs(d, exist_ok=True)
        derived = self._chi2_names()
        with open(root + ".paramnames", "w") as f:
            for n, lab in zip(self.names, self.labels):
                f.write(f"{n}\t{lab}\n")
            for n, lab in (self.like_derived.names if self.like_derived else []):
                f.write(f"{n}*\t{lab}\n")
            for n, lab in derived:
                f.write(f"{n}*\t{lab}\n")
        if ranges is not None:
            with open(root + ".ranges", "w") as f:
                for n, r in zip(self.names, ranges):
                    f.write(f"{n}\t{r[0]!r}\t{r[1]!r}\n")
                for n, _ in derived:                 # AddDerivedRange(name, mn=0) (ObjectParamNames.f90:480-508)
                    f.write(f"{n:<22}{fortran_e(0.0)}{'    N':<17}\n")
        if self.likelihoods:
            with open(root + ".likelihoods", "w") as f:
                for tag, typ, name, ver in self.likelihoods:
                    f.write("\t".join(str(x).strip() for x in ("1", typ, tag, name, ver)) + "\n")

    def _types(self):
        """likelihood types used more than once, in first-use order, with their members"""
        order, members = [], {}
        for i, (_, typ, _, _) in enumerate(self.likelihoods):
            if typ:
                if typ not in members:
                    order.append(typ)
                    members[typ] = []
                members[typ].append(i)
        return [(t, members[t]) for t in order if len(members[t]) > 1]

    def _chi2_names(self):
        if not self.likelihoods:
            return []
        lab = "\\chi^2_{\\rm %s}"                     # chisq_label, settings.f90:127
        out = [(f"chi2_{tag}", lab % tag.replace("_", "\\_")) for tag, _, _, _ in self.likelihoods]
        out.append(("chi2_prior", lab % "prior"))
        out += [(f"chi2_{t}", lab % t.replace("_", "\\_")) for t, _ in self._types()]
        return out

    def _derived(self, like, terms):
        """chi2 columns [steps, n_derived] from CurLike [steps] and terms [steps, n_like]"""
        cols = [2.0 * terms[:, i] for i in range(terms.shape[1])]
        cols.append(2.0 * (like - terms.sum(axis=1)))
        cols += [2.0 * terms[:, m].sum(axis=1) for _, m in self._types()]
        return np.stack(cols, axis=1)

    def _file(self, w):
        return f"{self.root}_{w + self.first_chain}.txt"

    def _emit(self, fh, point, weight):
        fh.write("".join(fortran_e(v, 16) for v in [float(weight), point[0], *point[1:]]) + "\n")

    def _move_done(self, fh, w, point, mult):
        """The chain leaves ``point`` after ``mult`` steps there (MoveDone with accpt)."""
        like = float(point[0])
        nacc = self.num_accept.get(w, 0)
        if like != LOGZERO and nacc > self.burn_in:               # MCMC.f90:177
            acc = self.acc.get(w, 0.0) + mult                      # SampleCollector.f90:97-104
            if acc >= self.thin or self.thin == 1:
                self._emit(fh, point, acc / self.thin)
                acc = math.fmod(acc, float(self.thin))
            self.acc[w] = acc
        self.num_accept[w] = nacc + 1
        best = self.max_like.get(w)
        if best is None or like < best[0]:                        # :182-185
            self.max_like[w] = (like, point.copy())

    def add_rows(self, rows, terms=None):
        """rows: [steps, n_used + 1, W] history block (params_used..., CurLike);
        terms: [steps, n_like, W] (history_terms) when writing chi2 columns."""
        rows = np.asarray(rows)
        steps, n1, W = rows.shape
        if self.likelihoods and (terms is None or np.shape(terms)[1] != len(self.likelihoods)):
            raise ValueError("chi2 columns need the per-likelihood history terms of every likelihood")
        walkers = range(W) if self.walkers is None else self.walkers
        dcols = self.like_derived.columns(rows[:, :n1 - 1, :]) if self.like_derived else None   # [steps, nd, W]
        for w in walkers:
            pts = np.concatenate([rows[:, n1 - 1:n1, w], rows[:, :n1 - 1, w]], axis=1)   # like, P...
            if dcols is not None:
                pts = np.concatenate([pts, dcols[:, :, w]], axis=1)
            if self.likelihoods:
                pts = np.concatenate([pts, self._derived(rows[:, n1 - 1, w], np.asarray(terms)[:, :, w])], axis=1)
            with open(self._file(w), "a") as fh:
                cur = self.pending.get(w)
                for t in range(steps):
                    p = pts[t]
                    if cur is not None and np.array_equal(cur[0], p):
                        cur[1] += 1
                    else:
                        if cur is not None:
                            self._move_done(fh, w, cur[0], cur[1])
                        cur = [p.copy(), 1]
                self.pending[w] = cur

    def append(self, sampler, first: int = None, count: int = None):
        """Write the history steps [first, first + count) of ``sampler``
        (default: everything recorded since the last call)."""
        total = sampler.history_count()
        if first is None:
            first = self.next_step if self.next_step is not None else 0
        if count is None:
            count = total - first
        if count > 0:
            terms = sampler.history_terms(first, count) if self.likelihoods else None
            self.add_rows(sampler.history_host(first, count), terms)
        self.next_step = first + max(count, 0)

    def _walkers(self, W):
        return list(range(W)) if self.walkers is None else list(self.walkers)

    def checkpoint_state(self, W: int) -> dict:
        """What a resume needs: the open weighted rows, the next history step
        and every chain file's length -- for every walker of the W-walker
        sampler, written or not -- so rows written after the checkpoint are cut
        off on resume and the files continue as if never interrupted."""
        return {"pending": {str(w): [np.asarray(c[0]).tolist(), int(c[1])]
                            for w, c in self.pending.items() if c is not None},
                "next_step": self.next_step,
                "num_accept": {str(w): n for w, n in self.num_accept.items()},
                "acc": {str(w): a for w, a in self.acc.items()},
                "max_like": {str(w): [b[0], np.asarray(b[1]).tolist()] for w, b in self.max_like.items()},
                "sizes": {str(w): (os.path.getsize(self._file(w)) if os.path.exists(self._file(w)) else 0)
                          for w in self._walkers(W)}}

    def restore(self, state: dict, W: int):
        sizes = state.get("sizes", {})
        for w in self._walkers(W):
            n = int(sizes.get(str(w), 0))
            f = self._file(w)
            if os.path.exists(f) and os.path.getsize(f) > n:
                with open(f, "r+b") as fh:
                    fh.truncate(n)
        self.pending = {int(w): [np.asarray(p, dtype=np.float64), c] for w, (p, c) in state["pending"].items()}
        self.next_step = state.get("next_step")
        self.num_accept = {int(w): int(n) for w, n in state.get("num_accept", {}).items()}
        self.acc = {int(w): float(a) for w, a in state.get("acc", {}).items()}
        self.max_like = {int(w): (float(b[0]), np.asarray(b[1], dtype=np.float64))
                         for w, b in state.get("max_like", {}).items()}

    def max_like_params(self, w):
        """(MaxLike, [like, P...]) of walker w: the best point it has moved off."""
        return self.max_like.get(w)

    def close(self):
        """End of the run: the points the chains sit at are not written
        (MoveDone writes a point only when the chain leaves it)."""
        self.pending = {}


class LikelihoodDerived:
    """The likelihoods' derived parameters for chain rows
    (addLikelihoodDerivedParams, GeneralTypes.f90:772-777:
    Derived(derived_indices) = derivedParameters(Theory, P(nuisance_indices))).

    likes: the LikelihoodList after add_nuisance_parameters; params_used: the
    1-based parameter indices of the history rows; P_fixed: the full parameter
    vector supplying the values of parameters that are not used (fixed)."""

    def __init__(self, likes, params_used, P_fixed, labels=None, device="cuda"):
        self.likes = [l for l in likes if getattr(l, "derived_names", None)]
        self.params_used = [int(i) for i in params_used]
        self.P_fixed = np.asarray(P_fixed, dtype=np.float64)
        self.device = device
        order = []
        for l in self.likes:
            for nm, ix in zip(l.derived_names, l.derived_indices):
                order.append((ix, nm))
        self.n = max([ix for ix, _ in order], default=0)
        names = [""] * self.n
        for ix, nm in order:
            names[ix - 1] = nm
        labels = labels or {}
        self.names = [(nm, labels.get(nm, nm)) for nm in names]

    def columns(self, P_used):
        """P_used [steps, n_used, W] -> derived [steps, n_derived, W] (device
        evaluation through cmbl_derived_batch)."""
        import torch
        steps, nu, W = P_used.shape
        full = np.broadcast_to(self.P_fixed, (steps, W, self.P_fixed.size)).copy()
        for k, i in enumerate(self.params_used):
            full[:, :, i - 1] = P_used[:, k, :]
        full = full.reshape(steps * W, -1)
        out = np.zeros((steps * W, self.n))
        for l in self.likes:
            nuis = torch.tensor(np.ascontiguousarray(full[:, [i - 1 for i in l.nuisance_indices]]), device=self.device)
            d = l.derived_batch(nuis).cpu().numpy()
            for k, ix in enumerate(l.derived_indices):
                out[:, ix - 1] = d[:, k]
        return out.reshape(steps, W, self.n).transpose(0, 2, 1)
