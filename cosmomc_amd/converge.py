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

from dataclasses import dataclass, field

import numpy as np


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
                                      min_sample_update: int | None = None) -> ConvergeResult:
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
        count = last - first + 1
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
                    res.converged = res.R < st.MPI_R_Stop and self.flukecheck
                    self.flukecheck = res.R < st.MPI_R_Stop
        if enough:
            # SampleCollector.f90:311-317 (Fortran precedence: .and. before .or.)
            res.update_proposal = st.MPI_LearnPropose and (
                M == 1 or ((st.covariance_is_diagonal or res.R < st.MPI_Max_R_ProposeUpdate)
                           and res.R > st.MPI_R_StopProposeUpdate))
        return res


def _device_of(provider):
    return getattr(provider, "device", "cuda")


def reference_window(count: int) -> tuple[int, int]:
    """0-based inclusive history rows of the reference's second-half window,
    Samples%Item(Count/2 : Count) (SampleCollector.f90:234-246)."""
    if count < 2:
        raise ValueError("need at least two samples")
    return count // 2 - 1, count - 1
