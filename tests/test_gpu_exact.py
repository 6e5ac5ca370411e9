"""CMBlikes like_approx = exact (unbinned full-sky ExactChiSq,
CMBlikes.f90:967-979 with the unbinned branch of CMBLikes_LogLike :1187-1206)
on the HIP kernel (cmbl_exact_kernel) vs the compiled reference
(tests/golden/exact_ref.json) and the numpy oracle.  GPU only.

The datasets are synthetic (cosmomc_amd.synthetic.make_exact, written by
oracle/gen_golden.py EXACT_CASES): the reference ships no unbinned dataset.

Tolerance: rtol 1e-10, atol 1e-8 on -lnL ~ 50..1300.  The kernel forms
tr(C^-1 Chat) and ln det from Cholesky factors where the reference uses an
eigendecomposition for C^-1/2; both are fp64 and the difference is rounding,
four orders inside the north star's |d lnL| < 1e-6.
"""
import numpy as np
import pytest

import cmblikes_oracle as co
import gen_golden as gg
from cosmomc_amd import synthetic as syn

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

EXACT = [c[0] for c in gg.EXACT_CASES]
RTOL, ATOL = 1e-10, 1e-8


def _open(path, overrides=None):
    from cosmomc_amd.likelihood import NativeCMBLikelihood
    return NativeCMBLikelihood("exact", path, overrides)


def _nuis(c, W):
    base = np.array(c["nuis"]).reshape(c["walkers"], -1)
    return base[np.arange(W) % len(base)]


@pytest.mark.parametrize("case", EXACT)
def test_exact_vs_reference_golden(exact_golden, exact_data, case):
    c = exact_golden["cases"][case]
    like = _open(exact_data[case])
    th = torch.tensor(syn.walker_theory(c["walkers"], seed=c["theory_seed"], lmax=c["lmax"], n_fields=6),
                      device="cuda")
    nu = torch.tensor(_nuis(c, c["walkers"]), device="cuda")
    got = like.loglike_batch(th, nu).cpu().numpy()
    np.testing.assert_allclose(got, c["minus_lnL"], rtol=RTOL, atol=ATOL)


@pytest.mark.parametrize("case", ["exact_TE_lowl", "exact_TEB_cal_aberration"])
@pytest.mark.parametrize("W", [1, 3, 4, 5, 64, 257])
def test_exact_walker_counts_vs_oracle(exact_golden, exact_data, case, W):
    c = exact_golden["cases"][case]
    like = _open(exact_data[case])
    o = co.CMBLikesOracle(exact_data[case], None, "exact")
    th = syn.walker_theory(W, seed=700 + W, lmax=c["lmax"], n_fields=6)
    nu = _nuis(c, W)
    got = like.loglike_batch(torch.tensor(th, device="cuda"), torch.tensor(nu, device="cuda")).cpu().numpy()
    idx = sorted({0, W // 2, W - 1})
    ref = np.array([o.loglike(th[w], nu[w]) for w in idx])
    np.testing.assert_allclose(got[idx], ref, rtol=RTOL, atol=ATOL)


def test_exact_padded_stride_and_shared_theory(exact_golden, exact_data):
    """Theory rows in a wider buffer (ld_field > lmax + 1, odd, extra fields),
    and ld_walker = 0 (every walker on one slow point)."""
    case = "exact_TEB_cal_aberration"
    c = exact_golden["cases"][case]
    like = _open(exact_data[case])
    W = 5
    th = syn.walker_theory(W, seed=c["theory_seed"], lmax=c["lmax"], n_fields=6)
    big = np.full((W, 10, c["lmax"] + 8), np.nan)
    big[:, :6, :c["lmax"] + 1] = th
    nu = _nuis(c, W)
    t_big = torch.tensor(big, device="cuda")[:, :, :c["lmax"] + 7]
    got = like.loglike_batch(t_big, torch.tensor(nu, device="cuda")).cpu().numpy()
    np.testing.assert_allclose(got[:4], c["minus_lnL"], rtol=RTOL, atol=ATOL)
    shared = torch.tensor(th[0], device="cuda").unsqueeze(0).expand(W, -1, -1)
    got = like.loglike_batch(shared, torch.tensor(nu, device="cuda")).cpu().numpy()
    o = co.CMBLikesOracle(exact_data[case], None, "exact")
    ref = np.array([o.loglike(th[0], nu[w]) for w in range(W)])
    np.testing.assert_allclose(got, ref, rtol=RTOL, atol=ATOL)


def test_exact_host_entry(exact_golden, exact_data):
    case = "exact_TE_lowl"
    c = exact_golden["cases"][case]
    like = _open(exact_data[case])
    th = syn.walker_theory(c["walkers"], seed=c["theory_seed"], lmax=c["lmax"], n_fields=6)
    got = like.loglike_host(th, np.zeros((c["walkers"], 0)))
    np.testing.assert_allclose(got, c["minus_lnL"], rtol=RTOL, atol=ATOL)


def test_exact_not_positive_definite_is_nan(exact_golden, exact_data):
    """A theory + noise matrix that is not positive definite: the reference's
    C^-1/2 raises a negative eigenvalue to -1/2 (NaN); the kernel returns NaN."""
    case = "exact_TE_lowl"
    c = exact_golden["cases"][case]
    like = _open(exact_data[case])
    th = syn.walker_theory(2, seed=c["theory_seed"], lmax=c["lmax"], n_fields=6)
    th[1, 1, 10] = 1e6                      # TE >> sqrt(TT EE) at l = 10
    got = like.loglike_batch(torch.tensor(th, device="cuda"), torch.zeros((2, 0), dtype=torch.float64,
                                                                            device="cuda")).cpu().numpy()
    assert np.isfinite(got[0]) and np.isnan(got[1])


@pytest.mark.parametrize("over,code", [({"binned": "T", "nbins": "3"}, -3),      # exact cannot be binned
                                       ({"like_approx": "gaussian"}, -6),          # unbinned gaussian
                                       ({"fields_use": "T E", "maps_use": "T"}, 0)])
def test_exact_loader_options(exact_data, over, code):
    from cosmomc_amd._native import NativeError
    path = exact_data["exact_TE_lowl"]
    if code == 0:
        assert _open(path, over).n_nuis == 0
        return
    with pytest.raises(NativeError) as e:
        _open(path, over)
    assert e.value.code == code
