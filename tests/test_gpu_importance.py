"""Importance sampling on the GPU (cosmomc_amd.importance.GPUEvaluator): a
text chain over (A, calPlanck) is re-weighted by plik_lite evaluated on the
theory A x base D_l (redo_theory: the theory function fills the registered
theory buffer for each batch of rows), bounds and the calPlanck prior, i.e.
GetLogLikePost (calclike.f90:334-354) per row.  The rows, weights and new
likelihoods match the C oracle's plik_lite (tests/test_oracle.py pins it to
the compiled reference) to rtol 1e-9."""
import numpy as np
import pytest

import pyoracle as po
from cosmomc_amd import synthetic as syn
from cosmomc_amd.chains import fortran_e
from cosmomc_amd.importance import GPUEvaluator, ImportanceSampler, ImportanceSettings, LOGZERO, read_chain_rows

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("temperature", [1.0, 2.0])
def test_importance_plik_theory_batches(tmp_path, temperature):
    from cosmomc_amd.likelihood import NativeCMBLikelihood
    from cosmomc_amd.sampler import BatchedMCMC
    data = syn.make_plik_lite(12345)
    like = NativeCMBLikelihood("PLIK_LITE", data.write(str(tmp_path)))
    like.nuisance_indices = [2]
    W, n = 32, 75                                     # 75 rows: two full batches and a padded one
    base_np = np.ascontiguousarray(syn.base_theory(2508)[:3])
    base = torch.tensor(base_np, device="cuda")
    theory = base.unsqueeze(0).repeat(W, 1, 1).contiguous()
    pmin, pmax = np.array([0.9, 0.9]), np.array([1.1, 1.1])
    pm, ps = np.array([0.0, 1.0]), np.array([0.0, 0.0025])
    s = BatchedMCMC(W, 2, [1, 2], [[1], [2]], 1, pmin, pmax, pm, ps, temperature=temperature)
    s.set_covariance(np.diag([1e-6, 1e-6]))
    s.add_likelihood(like, theory)

    def theory_fn(P):
        A = torch.tensor(P[:, 0], device="cuda").reshape(-1, 1, 1)
        theory.copy_(base.unsqueeze(0) * A)
    g = syn.gaussians(77, 3 * n).reshape(n, 3)
    A = 1.0 + 0.004 * g[:, 0]
    cal = 1.0 + 0.0025 * g[:, 1]
    A[7] = 1.2                                        # outside the new bounds: weight 0
    orc = po.PlikLite(data)

    def truth(Pr):
        out = np.empty(Pr.shape[0])
        for k, (a, c) in enumerate(Pr):
            if np.any(Pr[k] > pmax) or np.any(Pr[k] < pmin):
                out[k] = LOGZERO
            else:
                out[k] = (orc.loglike(a * base_np, c) + 0.5 * ((c - 1.0) / 0.0025) ** 2) / temperature
        return out
    old = truth(np.column_stack([A, cal]))
    old[7] = 50.0
    like_in = old + 0.3 * g[:, 2]                     # the "old" chain's -lnL
    mult = 1.0 + (np.arange(n) % 3)
    with open(tmp_path / "in.txt", "w") as f:
        for k in range(n):
            f.write("".join(fortran_e(v) for v in (mult[k], like_in[k], A[k], cal[k])) + "\n")
    st = ImportanceSettings(redo_likelihoods=True, redo_theory=True, redo_skip=0, redo_auto_likescale=False)
    r = ImportanceSampler(st, [1, 2], np.array([1.0, 1.0]), GPUEvaluator(s, theory_fn)).run(
        str(tmp_path / "in.txt"), str(tmp_path / "post"))
    chain = read_chain_rows(str(tmp_path / "in.txt"))
    tl = truth(chain[:, 2:])
    w = np.where(tl == LOGZERO, 0.0, np.exp(chain[:, 1] - tl))
    keep = chain[:, 0] * w > 1e-100
    assert keep.sum() == n - 1 and len(r.rows) == n - 1
    got_m = np.array([m for m, _, _ in r.rows])
    got_t = np.array([t for _, t, _ in r.rows])
    np.testing.assert_allclose(got_t, tl[keep], rtol=1e-9)
    np.testing.assert_allclose(got_m, (chain[:, 0] * w)[keep], rtol=1e-8)
    assert r.mult_ratio == pytest.approx(w.sum(), rel=1e-8)
    assert r.num_used == n - 1                        # the out-of-bounds row is skipped (CheckPriorCuts)
    assert r.weight_min == pytest.approx(w[keep].min(), rel=1e-8)
