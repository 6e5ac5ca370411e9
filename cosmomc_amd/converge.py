"""Convergence test and proposal learning across every walker on every GPU.

Mirrors ``TMpiChainCollector_UpdateCovAndCheckConverge``
(source/SampleCollector.f90:212-322) and ``GelmanRubinEvalues``
(source/samples.f90:41-67).  In the reference each MPI rank is one chain and
the ranks ``MPI_ALLGATHER`` their second-half mean/covariance; here every
walker is a chain, each GPU reduces its own walkers on device
(``cmbs_chain_moments``, a fixed-order HIP reduction) and the GPUs combine
the partial sums with two small ``all_reduce`` calls (RCCL over xGMI on the
GPU box, gloo in the CPU tests):

  pass 1: [sum count, sum count*mean, sum count*cov, sum cov, chains]
          -> pooled mean, MPICovMat, mean of covariances
  pass 2: sum count*(mean - pooled)(mean - pooled)^T
          -> covariance of chain means (x M/(M-1))

Two passes keep the covariance of the means free of the cancellation a
one-pass sum of squares would have.  The n_used x n_used eigenproblem is
solved on the host, as in the reference.
"""
from __future__ import annotations

import warnings
from dataclasses import dataclass, field

import numpy as np


def _real4(x: float) -> float:
    """The value a Fortran default REAL holds (TMPIData's MPI_R_Stop etc. are REAL(4))."""
    return float(np.float32(x))


@dataclass
class CollectorSettings:
    """TMPIData defaults (SampleCollector.f90:12-35) and their ini keys (:115-127)."""
    MPI_R_Stop: float = 0.05                  # MPI_Converge_Stop
    MPI_Min_Sample_Update: int = 200
    MPI_Sample_update_freq: int = 40
    MPI_LearnPropose: bool = True
    MPI_Max_R_ProposeUpdate: float = 2.0
    MPI_Max_R_ProposeUpdateNew: float = 30.0
    MPI_R_StopProposeUpdate: float = 0.0
    MPI_Check_Limit_Converge: bool = False
    MPI_Limit_Converge: float = 0.025
    MPI_Limit_Converge_Err: float = 0.3
    MPI_Limit_Param: int = 0                  # full parameter index; 0 = every used parameter
    covariance_is_diagonal: bool = False      # BaseParams%covariance_is_diagonal

    @classmethod
    def from_ini(cls, ini) -> "CollectorSettings":
        s = cls()
        s.MPI_R_Stop = float(ini.get("MPI_Converge_Stop", s.MPI_R_Stop))
        s.MPI_LearnPropose = str(ini.get("MPI_LearnPropose", "T")).upper().startswith("T")
        if s.MPI_LearnPropose:
            s.MPI_R_StopProposeUpdate = float(ini.get("MPI_R_StopProposeUpdate", s.MPI_R_StopProposeUpdate))
            s.MPI_Max_R_ProposeUpdate = float(ini.get("MPI_Max_R_ProposeUpdate", s.MPI_Max_R_ProposeUpdate))
            s.MPI_Max_R_ProposeUpdateNew = float(ini.get("MPI_Max_R_ProposeUpdateNew",
                                                         s.MPI_Max_R_ProposeUpdateNew))
        s.MPI_Check_Limit_Converge = str(ini.get("MPI_Check_Limit_Converge", "F")).upper().startswith("T")
        if s.MPI_Check_Limit_Converge:
            s.MPI_Limit_Converge = float(ini.get("MPI_Limit_Converge", s.MPI_Limit_Converge))
            s.MPI_Limit_Converge_Err = float(ini.get("MPI_Limit_Converge_Err", s.MPI_Limit_Converge_Err))
            s.MPI_Limit_Param = int(ini.get("MPI_Limit_Param", s.MPI_Limit_Param))
        return s


@dataclass
class ConvergeResult:
    R: float                         # R-1 (largest Gelman-Rubin eigenvalue); 1e6 if not invertible
    evals: np.ndarray | None
    mean: np.ndarray
    propose_cov: np.ndarray          # MPICovMat: count-weighted mean of the chain covariances
    cov: np.ndarray                  # plain mean of the chain covariances
    meanscov: np.ndarray             # covariance of the chain means x M/(M-1)
    n_chains: int
    enough_samples: bool
    converged: bool = False
    update_proposal: bool = False
    extras: dict = field(default_factory=dict)


def gelman_rubin_evalues(cov: np.ndarray, meanscov: np.ndarray):
    """(ok, evals): diagonal-normalise both matrices by sqrt(diag(cov)),
    L = chol(cov'), evals of L^-1 meanscov' L^-T (samples.f90:41-67)."""
    sc = np.sqrt(np.diag(cov))
    rot = cov / sc[:, None] / sc[None, :]
    rm = meanscov / sc[:, None] / sc[None, :]
    try:
        L = np.linalg.cholesky(rot)
    except np.linalg.LinAlgError:
        return False, None
    Li = np.linalg.inv(L)
    Li = np.tril(Li)                        # Matrix_CholeskyRootInverse zeroes the upper triangle
    B = Li @ rm @ Li.T
    return True, np.linalg.eigvalsh(0.5 * (B + B.T))


def _all_reduce(t, group):
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


class ConvergenceExchange:
    """The periodic exchange of TMpiChainCollector across GPUs.

    ``provider.chain_moments(first, last, gmean=None)`` returns this rank's
    partial sums as a torch tensor (device tensor from ``BatchedMCMC``; the
    collective runs on whatever device it lives on)."""

    def __init__(self, n_used: int, settings: CollectorSettings | None = None, group=None):
        self.n = n_used
        self.settings = settings or CollectorSettings()
        self.group = group
        self.flukecheck = False

    def update_cov_and_check_converge(self, provider, first: int, last: int,
                                      min_sample_update: int | None = None,
                                      window_count: int | None = None) -> ConvergeResult:
        """window_count: the smallest per-chain window size when the chains'
        windows differ (ChainCollector); else last - first + 1."""
        import torch
        n, st = self.n, self.settings
        p1 = _all_reduce(provider.chain_moments(first, last), self.group)
        p1 = p1.double().cpu().numpy()
        norm = p1[0]
        mean = p1[1:1 + n] / norm
        propose_cov = p1[1 + n:1 + n + n * n].reshape(n, n) / norm
        M = int(round(p1[1 + n + 2 * n * n]))
        cov = p1[1 + n + n * n:1 + n + 2 * n * n].reshape(n, n) / M
        g = torch.as_tensor(mean, dtype=torch.float64, device=_device_of(provider))
        p2 = _all_reduce(provider.chain_moments(first, last, g), self.group).double().cpu().numpy()
        meanscov = p2.reshape(n, n) / norm
        count = last - first + 1 if window_count is None else window_count
        msu = st.MPI_Min_Sample_Update if min_sample_update is None else min_sample_update
        enough = count > msu // 2 + 2                       # all(MPIMeans(0,:) > Min/2 + 2)
        res = ConvergeResult(R=1e6, evals=None, mean=mean, propose_cov=0.5 * (propose_cov + propose_cov.T),
                             cov=0.5 * (cov + cov.T), meanscov=None, n_chains=M, enough_samples=enough)
        if M > 1:
            meanscov = meanscov * M / (M - 1)
            res.meanscov = 0.5 * (meanscov + meanscov.T)
            ok, ev = gelman_rubin_evalues(res.cov, res.meanscov)
            if ok:
                res.evals = ev
                res.R = float(ev.max())
                if enough:
                    res.converged = res.R < _real4(st.MPI_R_Stop) and self.flukecheck
                    self.flukecheck = res.R < _real4(st.MPI_R_Stop)
        if enough:
            # SampleCollector.f90:311-317 (Fortran precedence: .and. before .or.)
            res.update_proposal = st.MPI_LearnPropose and (
                M == 1 or ((st.covariance_is_diagonal or res.R < _real4(st.MPI_Max_R_ProposeUpdate))
                           and res.R > _real4(st.MPI_R_StopProposeUpdate)))
        return res


def _device_of(provider):
    return getattr(provider, "device", "cuda")


def reference_window(count: int) -> tuple[int, int]:
    """0-based inclusive history rows of the reference's second-half window,
    Samples%Item(Count/2 : Count) (SampleCollector.f90:234-246)."""
    if count < 2:
        raise ValueError("need at least two samples")
    return count // 2 - 1, count - 1


class ChainCollector:
    """TMpiChainCollector_AddNewPoint / UpdateCovAndCheckConverge
    (SampleCollector.f90:212-460) for every walker of every rank: each walker
    is one chain with its own Samples list (cmbs_collector_* on device).

    Per processed block of history steps: AddNewPoint at every output_thin-th
    step (MCMC.f90:147; output_thin = oversample_fast for the Metropolis
    sampler, 1 for fast dragging, :235, :460); burn-in per walker; when
    walker 0 (global; "rank 0") burns, MPI_Sample_update_freq *= num_params_used
    (num_slow when dragging) and every chain's MPI_Min_Sample_Update becomes
    50 + 4 num_slow + num_fast, + 4 num_fast (x oversample_fast when dragging)
    (:391-404); all_burn = every walker on every rank burned (the ISEND/IRECV
    barrier of :380-389 as an all-reduce); DoUpdates once all_burn and Count >=
    Min + 1; then walker 0 triggers an exchange whenever its Count is a
    multiple of the update frequency (:429-446) and the exchange runs once every
    chain can answer (DoUpdates everywhere).  The block length the host should
    step next is ``next_block()``: it ends exactly at walker 0's next trigger.

    Chains are stepped in lock step, so every chain enters the exchange at the
    same step; in the reference each rank enters when the trigger reaches it,
    a few samples apart -- a timing the reference itself does not fix."""

    def __init__(self, sampler, settings: CollectorSettings | None = None, num_slow: int = 0, num_fast: int = 0,
                 dragging: bool = False, oversample_fast: int = 1, output_thin: int | None = None, group=None,
                 sample_capacity: int | None = None, thin_limit: int | None = None, root: str | None = None):
        self.s = sampler
        self.settings = settings or CollectorSettings()
        self.n = len(sampler.params_used)
        self.num_slow, self.num_fast = num_slow, num_fast
        self.dragging = dragging
        self.oversample_fast = max(1, oversample_fast)
        self.output_thin = output_thin if output_thin is not None else (1 if dragging else self.oversample_fast)
        self.group = group
        self.root = root
        cap = sample_capacity or getattr(sampler, "_hist_cap", 0)
        # Samples%Thin(2) once a list passes the reference's 500000 (SampleCollector.f90:300-304), or half
        # the list capacity when that is smaller, so a long run thins and goes on instead of overflowing.
        # The items are history steps: the ring must still hold the second half of each list's window.
        self.thin_limit = min(500000, max(1, cap // 2)) if thin_limit is None else thin_limit
        if thin_limit is None and self.thin_limit < 500000:
            # a known divergence from the reference, chosen here rather than by the caller: its
            # lists thin at 500000 items whatever their length; R-1 and the learnt proposals
            # differ once a list passes this limit (an explicit thin_limit is the caller's choice)
            warnings.warn(f"ChainCollector: lists are thinned at {self.thin_limit} items (history capacity "
                          f"{cap}), not at the reference's 500000 (SampleCollector.f90:300-304); size "
                          f"sample_capacity >= 1000000 to thin where the reference does", stacklevel=2)
        sampler.collector_enable(cap)
        self.cap = cap
        self.min_update = self.settings.MPI_Min_Sample_Update
        self.update_freq = self.settings.MPI_Sample_update_freq
        self.min_after_burn = 50 + 4 * num_slow + num_fast
        if dragging:
            self.min_after_burn *= self.oversample_fast
        else:
            self.min_after_burn += 4 * num_fast
        self.next_step = 0
        self.burn0 = False
        self.all_burn = False
        self.waiting = False
        self.done = False
        self.count0 = 0
        self.min_count = 0
        self.exchange = ConvergenceExchange(self.n, self.settings, group)
        self.results: list[ConvergeResult] = []
        import torch.distributed as dist
        self._world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self._rank = dist.get_rank(group) if self._world > 1 else 0

    _STATE = ("next_step", "burn0", "all_burn", "waiting", "done", "count0", "min_count", "update_freq",
              "min_update")

    def checkpoint_state(self) -> dict:
        """The host side of the collector a resume needs (the Samples lists
        themselves are in the sampler's device image): the next history step
        to add, walker 0's burn-in and trigger state, all_burn, the update
        frequency and MPI_Min_Sample_Update in force and flukecheck -- the
        pieces TMpiChainCollector_SaveState writes (SampleCollector.f90:139-151)."""
        st = {k: getattr(self, k) for k in self._STATE}
        st["flukecheck"] = bool(self.exchange.flukecheck)
        st["cap"] = self.cap
        return st

    def restore(self, state: dict):
        """Undo checkpoint_state (TMpiChainCollector_ReadState, :153-172)."""
        if int(state.get("cap", self.cap)) != self.cap:
            raise ValueError(f"checkpointed collector capacity {state['cap']} != {self.cap}")
        for k in self._STATE:
            setattr(self, k, type(getattr(self, k))(state[k]))
        self.exchange.flukecheck = bool(state["flukecheck"])

    # -- cross-rank reductions of the per-walker collector state
    def _reduce(self, burned, total, count0, mincount):
        import torch
        if self._world == 1:
            return burned, total, count0, mincount
        import torch.distributed as dist
        dev = "cuda" if torch.cuda.is_available() and dist.get_backend(self.group) == "nccl" else "cpu"
        a = torch.tensor([burned, total, count0], dtype=torch.float64, device=dev)
        dist.all_reduce(a, op=dist.ReduceOp.SUM, group=self.group)
        b = torch.tensor([mincount], dtype=torch.float64, device=dev)
        dist.all_reduce(b, op=dist.ReduceOp.MIN, group=self.group)
        return int(a[0].item()), int(a[1].item()), int(a[2].item()), int(b[0].item())

    def next_block(self) -> int:
        """History steps to run before the next ``process`` call: up to walker
        0's next trigger once it can trigger, else one update period."""
        if self.burn0 and self.all_burn and not self.waiting and self.count0 >= self.min_update + 1:
            k = self.update_freq - self.count0 % self.update_freq
            return max(1, k) * self.output_thin
        return max(1, self.update_freq) * self.output_thin

    def process(self) -> ConvergeResult | None:
        """AddNewPoint for every history step recorded since the last call, then
        the exchange if one is due.  Returns its ConvergeResult (or None)."""
        s = self.s
        total_steps = s.history_count()
        steps = [t for t in range(self.next_step, total_steps) if (t + 1) % self.output_thin == 0]
        self.next_step = total_steps
        s.collector_add(steps, self.min_after_burn, check_burn=True)
        _, count, burn, _ = s.collector_state()
        c0 = int(count[0]) if self._rank == 0 else 0
        b0 = int(burn[0]) if self._rank == 0 else 0
        burned, total, c0, minc = self._reduce(int(burn.sum()), s.W, c0, int(count.min()))
        b0 = self._reduce(b0, 0, 0, 0)[0] if self._world > 1 else b0
        self.count0, self.min_count = c0, minc
        if b0 and not self.burn0:                  # walker 0's own burn (:391-404)
            self.burn0 = True
            self.update_freq *= self.num_slow if self.dragging else self.n
            self.min_update = self.min_after_burn
        if not self.all_burn and burned == total:
            self.all_burn = True
        do0 = self.all_burn and self.count0 >= self.min_update + 1
        if do0 and not self.waiting and self.count0 % max(1, self.update_freq) == 0:
            self.waiting = True                     # rank 0's ISSEND trigger (:436-441)
        if not (self.waiting and self.all_burn and self.min_count >= self.min_update + 1):
            return None
        self.waiting = False
        return self._update_cov_and_check_converge()

    def _update_cov_and_check_converge(self) -> ConvergeResult:
        st = self.settings
        wc = self.min_count - self.min_count // 2 + 1
        prov = _CollectorMoments(self.s)
        res = self.exchange.update_cov_and_check_converge(prov, 0, 0, self.min_update, window_count=wc)
        if res.converged and st.MPI_Check_Limit_Converge:
            ok, worst, _ = self.check_limits(res.propose_cov)
            res.extras["limit_err"] = worst
            res.converged = ok
        self.done = self.done or res.converged
        if res.evals is not None:                   # Samples%Thin(2), MPI_thin_fac * 2 where Count > 500000
            self.s.collector_thin(self.thin_limit)   # (:300-304; per walker on device)
        if self.root and self._rank == 0:           # ConvergeStatus (:461-475)
            with open(self.root + ".converge_stat", "w") as f:
                f.write(f"{res.R!r}\n" + ("Done\n" if res.converged else ""))
        self.results.append(res)
        return res

    def check_limits(self, propose_cov):
        """CheckLimitsConverge: every chain's ConfidVal limits (device), all
        gathered, against the pooled standard deviations."""
        import torch
        st = self.settings
        if st.MPI_Limit_Param:
            params = [self.s.params_used.index(st.MPI_Limit_Param)]
        else:
            params = list(range(self.n))
        lim = self.s.collector_limits(params, st.MPI_Limit_Converge)
        if self._world > 1:
            import torch.distributed as dist
            if dist.get_backend(self.group) != "nccl":
                lim = lim.cpu()
            parts = [torch.empty_like(lim) for _ in range(self._world)]
            dist.all_gather(parts, lim, group=self.group)
            lim = torch.cat(parts)
        lim = lim.double().cpu().numpy()
        M = lim.shape[0]
        mean_lim = lim.sum(axis=0) / M
        var = ((lim - mean_lim[None]) ** 2).sum(axis=0) / (M - 1)
        err = np.sqrt(var / np.diag(propose_cov)[params][:, None])
        worst = float(err.max())
        return worst < _real4(st.MPI_Limit_Converge_Err), worst, err


class _CollectorMoments:
    """chain_moments provider over each walker's own collector window."""

    def __init__(self, sampler):
        self.s = sampler
        self.device = getattr(sampler, "device", "cuda")

    def chain_moments(self, first, last, gmean=None):
        return self.s.collector_moments(gmean)
