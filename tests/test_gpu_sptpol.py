"""SPTpol TE/EE 2017 and BB 2019 HIP kernels vs the compiled reference (golden
fixtures, synthetic datasets in the reference's on-disk formats) and the
numpy oracle.  GPU only, through the C ABI.

Tolerance (fp64): rtol 1e-10.  The GPU sums the window contractions in MFMA
order and forms the chi^2 with the explicit inverse covariance instead of
dpotrs; -lnL is O(10-1000), so |d lnL| stays below 1e-7, inside the north
star's 1e-6.
"""
import numpy as np
import pytest

import sptpol_oracle as so
from conftest import load_golden, sptpol_overrides
from cosmomc_amd import synthetic as syn

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

CASES = list(load_golden("sptpol_ref.json")["cases"])
RTOL, ATOL = 1e-10, 1e-8


def _nf(tag):
    return 3 if tag == "SPTPOL_TEEE" else 6


def _open(c, ds):
    from cosmomc_amd.likelihood import NativeCMBLikelihood
    return NativeCMBLikelihood(c["tag"], ds, sptpol_overrides(c, ds))


@pytest.mark.parametrize("case", CASES)
def test_sptpol_vs_reference_golden(sptpol_golden, sptpol_data, case):
    c = sptpol_golden["cases"][case]
    ds = sptpol_data[c["tag"]]
    like = _open(c, ds)
    th = syn.walker_theory(c["walkers"], seed=c["theory_seed"], lmax=c["lmax"], n_fields=_nf(c["tag"]))
    got = like.loglike_batch(torch.tensor(th, device="cuda"),
                             torch.tensor(c["nuis"], dtype=torch.float64, device="cuda")).cpu().numpy()
    np.testing.assert_allclose(got, c["minus_lnL"], rtol=RTOL, atol=ATOL)


@pytest.mark.parametrize("case", ["teee_aberration_priors", "bb_priors_blind_abb"])
@pytest.mark.parametrize("W", [1, 64, 65, 200])
def test_sptpol_walker_counts_vs_oracle(sptpol_golden, sptpol_data, case, W):
    c = sptpol_golden["cases"][case]
    ds = sptpol_data[c["tag"]]
    like = _open(c, ds)
    o = so.open_sptpol(c["tag"], ds, sptpol_overrides(c, ds))
    th = syn.walker_theory(W, seed=7 + W, lmax=c["lmax"], n_fields=_nf(c["tag"]))
    base = np.array(c["nuis"])
    nu = base[np.arange(W) % len(base)] * (1.0 + 1e-3 * np.cos(np.arange(W)))[:, None]
    got = like.loglike_batch(torch.tensor(th, device="cuda"), torch.tensor(nu, device="cuda")).cpu().numpy()
    idx = sorted(set([0, W - 1, W // 2, min(W - 1, 64)]))
    ref = o.loglike_batch(th[idx], nu[idx])
    np.testing.assert_allclose(got[idx], ref, rtol=RTOL, atol=ATOL)


@pytest.mark.parametrize("tag", ["SPTPOL_TEEE", "SPTPOL_BB"])
def test_sptpol_padded_unaligned_and_shared_theory(sptpol_golden, sptpol_data, tag):
    """Odd ld_field (scalar theory loads), padded rows, strided nuisance rows,
    and ld_walker = 0 (every walker on one cached slow point)."""
    from cosmomc_amd import _native as N
    c = next(v for v in sptpol_golden["cases"].values() if v["tag"] == tag and not v["overrides"])
    ds = sptpol_data[tag]
    like = _open(c, ds)
    o = so.open_sptpol(tag, ds)
    W, nf = 5, _nf(tag)
    th = syn.walker_theory(W, seed=c["theory_seed"], lmax=c["lmax"], n_fields=nf)
    ldf = c["lmax"] + 6                      # odd row length
    big = np.zeros((W, nf, ldf))
    big[:, :, :c["lmax"] + 1] = th
    nn = len(c["nuis"][0])
    nu = np.zeros((W, nn + 3))
    nu[:, :nn] = np.array(c["nuis"])[np.arange(W) % len(c["nuis"])]
    dl = torch.tensor(big, device="cuda")
    nut = torch.tensor(nu, device="cuda")
    out = torch.zeros(W, dtype=torch.float64, device="cuda")
    rc = N.lib().cmbl_loglike_batch(like.handle, W, dl.data_ptr(), ldf, nf * ldf, nut.data_ptr(), nn + 3,
                                    out.data_ptr(), None, None)
    assert rc == 0, like.last_error() if hasattr(like, "last_error") else rc
    torch.cuda.synchronize()
    np.testing.assert_allclose(out.cpu().numpy(), o.loglike_batch(th, nu[:, :nn]), rtol=RTOL, atol=ATOL)
    # shared theory: walker 0's row for everybody
    rc = N.lib().cmbl_loglike_batch(like.handle, W, dl.data_ptr(), ldf, 0, nut.data_ptr(), nn + 3,
                                    out.data_ptr(), None, None)
    assert rc == 0
    torch.cuda.synchronize()
    ref = o.loglike_batch(np.repeat(th[:1], W, axis=0), nu[:, :nn])
    np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=RTOL, atol=ATOL)


def test_sptpol_theory_beyond_lmax_is_ignored(sptpol_golden, sptpol_data):
    """Rows longer than lmax+1 holding NaN past lmax+1 (ClArray reads dls(1:lmax+1)
    only): the result is unchanged."""
    c = sptpol_golden["cases"]["teee_default"]
    ds = sptpol_data["SPTPOL_TEEE"]
    like = _open(c, ds)
    th = syn.walker_theory(c["walkers"], seed=c["theory_seed"], lmax=c["lmax"], n_fields=3)
    big = np.full((c["walkers"], 3, c["lmax"] + 64), np.nan)
    big[:, :, :c["lmax"] + 1] = th
    got = like.loglike_batch(torch.tensor(big, device="cuda"),
                             torch.tensor(c["nuis"], dtype=torch.float64, device="cuda")).cpu().numpy()
    np.testing.assert_allclose(got, c["minus_lnL"], rtol=RTOL, atol=ATOL)
