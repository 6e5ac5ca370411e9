"""SMICA (TSmica_planck, source/CMBlikes.f90:1262-1339) through the C ABI vs
the compiled reference (tests/golden/smica_ref.json, oracle/gen_golden.py
gen_smica) and the numpy oracle.  GPU only.

The reference ships no SMICA dataset: cosmomc_amd.synthetic.make_smica writes
a binned TT CMBLike2 dataset with the SMICA nuisance_params (five foreground
parameters, a calibration, the derived D_l(2000)).  The foreground is added to
the TT map spectra in window staging (cmbl_smica_prologue + cmbl_window_kernel);
the derived parameter comes from cmbl_derived_batch.

Tolerances (fp64): gaussian rtol 1e-10, HL rtol 1e-9 (as tests/test_gpu_cmblikes.py);
derived rtol 1e-13 (one exp and one pow per walker: the device's and glibc's
libm may differ in the last bit).
"""
import numpy as np
import pytest

import cmblikes_oracle as co
from cosmomc_amd import synthetic as syn

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

CASES = ["smica_gauss", "smica_gauss_run", "smica_gauss_calname", "smica_hl_aber_calname", "smica_calparam_override",
         "smica_calname_unknown"]


def _open(smica_data, c):
    from cosmomc_amd.likelihood import NativeCMBLikelihood
    return NativeCMBLikelihood("SMICA", smica_data[c["like_approx"]], c["overrides"])


def _tol(c):
    return (1e-9, 1e-8) if c["like_approx"] == "HL" else (1e-10, 1e-9)


@pytest.mark.parametrize("case", CASES)
def test_smica_vs_reference_golden(smica_golden, smica_data, case):
    c = smica_golden["cases"][case]
    like = _open(smica_data, c)
    th = torch.tensor(syn.walker_theory(c["walkers"], seed=c["theory_seed"], lmax=c["lmax"], n_fields=6),
                      device="cuda")
    nu = torch.tensor(c["nuis"], dtype=torch.float64, device="cuda")
    got = like.loglike_batch(th, nu).cpu().numpy()
    rtol, atol = _tol(c)
    np.testing.assert_allclose(got, c["minus_lnL"], rtol=rtol, atol=atol)
    der = like.derived_batch(nu).cpu().numpy()
    np.testing.assert_allclose(der, np.array(c["derived"]), rtol=1e-13, atol=0)
    assert like.status() == 0


@pytest.mark.parametrize("case", ["smica_gauss_calname", "smica_hl_aber_calname"])
@pytest.mark.parametrize("W", [1, 63, 64, 65, 257])
def test_smica_walker_counts_vs_oracle(smica_golden, smica_data, case, W):
    """W = 1..257 against the numpy oracle (pinned to the same goldens on CPU)."""
    c = smica_golden["cases"][case]
    like = _open(smica_data, c)
    o = co.CMBLikesOracle(smica_data[c["like_approx"]], c["overrides"], "SMICA")
    th = syn.walker_theory(W, seed=77 + W, lmax=c["lmax"], n_fields=6)
    base = np.array(c["nuis"])
    nu = base[np.arange(W) % len(base)].copy()
    nu[:, 2] += 0.01 * np.arange(W) / W              # every walker its own running index
    got = like.loglike_batch(torch.tensor(th, device="cuda"), torch.tensor(nu, device="cuda")).cpu().numpy()
    idx = sorted(set([0, W - 1, W // 2, min(W - 1, 64)]))
    ref = np.array([o.loglike(th[w], nu[w]) for w in idx])
    rtol, atol = _tol(c)
    np.testing.assert_allclose(got[idx], ref, rtol=rtol, atol=atol)
    der = like.derived_batch(torch.tensor(nu, device="cuda")).cpu().numpy()
    np.testing.assert_allclose(der[idx], np.array([o.derived(nu[w]) for w in idx]), rtol=1e-13, atol=0)


def test_smica_strided_theory_and_nuisance(smica_golden, smica_data):
    """Padded theory rows, a shared theory row (ld_walker = 0) and a strided
    nuisance block."""
    c = smica_golden["cases"]["smica_gauss_calname"]
    like = _open(smica_data, c)
    o = co.CMBLikesOracle(smica_data["gaussian"], c["overrides"], "SMICA")
    W = 11
    th = syn.walker_theory(1, seed=5, lmax=c["lmax"], n_fields=6)
    big = np.zeros((1, 10, 2560))
    big[:, :6, :c["lmax"] + 1] = th
    nu = np.zeros((W, 9))
    nu[:, 2:8] = np.array(c["nuis"])[np.arange(W) % 4]
    tb = torch.tensor(big, device="cuda").expand(W, 10, 2560)
    got = like.loglike_batch(tb, torch.tensor(nu, device="cuda")[:, 2:8]).cpu().numpy()
    ref = [o.loglike(th[0], nu[w, 2:8]) for w in range(W)]
    np.testing.assert_allclose(got, ref, rtol=1e-10)


def test_smica_metadata_and_refusals(smica_data, tmp_path):
    from cosmomc_amd import _native as N
    from cosmomc_amd.likelihood import LikelihoodList, NativeCMBLikelihood
    like = NativeCMBLikelihood("SMICA", smica_data["gaussian"], {"calibration_paramname": "cal_smica"})
    assert like.nuisance_names == [n for n, _ in syn.SMICA_PARAMS]
    assert like.derived_names == ["Dl2000_smica"]
    assert like.cl_lmax[0][0] == 2508
    ll = LikelihoodList()
    ll.add(like)
    names = ll.add_nuisance_parameters(["omegabh2"])
    assert names[1:] == like.nuisance_names and like.nuisance_indices == list(range(2, 8))
    assert like.derived_indices == [1]
    # exact + SMICA foregrounds, or the 5 foreground parameters missing: refused loudly
    with pytest.raises(N.NativeError):
        NativeCMBLikelihood("SMICA", smica_data["gaussian"], {"like_approx": "exact", "binned": "F"})
    p = tmp_path / "short.paramnames"
    p.write_text("A1_smica A_1\nn1_smica n_1\n")
    with pytest.raises(N.NativeError):
        NativeCMBLikelihood("SMICA", smica_data["gaussian"], {"nuisance_params": str(p)})
    # the same dataset opened as plain CMBlikes has no foreground: -lnL differs
    plain = NativeCMBLikelihood("smica_as_cmblikes", smica_data["gaussian"], {})
    assert plain.derived_names == [] and plain.nuisance_names == []
    th = torch.tensor(syn.walker_theory(2, lmax=2508, n_fields=6), device="cuda")
    nu = torch.tensor([list(syn.SMICA_FG) + [1.0]] * 2, dtype=torch.float64, device="cuda")
    a = like.loglike_batch(th, nu).cpu().numpy()
    b = plain.loglike_batch(th, nu[:, :0]).cpu().numpy()
    assert np.all(np.abs(a - b) > 1e-3)


def test_smica_fast_chain_and_chain_files(smica_data, tmp_path):
    """A SMICA fast-parameter chain (the five foreground parameters and the
    calibration in one fast block) on one cached theory: the walkers' terms
    at their final points are the oracle's, and the chain files carry the
    likelihood's derived D_l(2000) column (addLikelihoodDerivedParams,
    GeneralTypes.f90:772-777) before the chi2 columns."""
    from cosmomc_amd.chains import ChainWriter, LikelihoodDerived
    from cosmomc_amd.likelihood import LikelihoodList, NativeCMBLikelihood
    from cosmomc_amd.sampler import BatchedMCMC
    over = {"calibration_paramname": "cal_smica"}
    like = NativeCMBLikelihood("SMICA", smica_data["gaussian"], over)
    ll = LikelihoodList()
    ll.add(like)
    names = ll.add_nuisance_parameters([])
    assert like.nuisance_indices == [1, 2, 3, 4, 5, 6]
    W, steps = 128, 30
    P0 = np.array(list(syn.SMICA_FG) + [1.0])
    width = np.array([3.0, 0.05, 0.1, 2.0, 0.05, 0.0025])
    pmin, pmax = P0 - 20 * width, P0 + 20 * width
    used = [1, 2, 3, 4, 5, 6]
    s = BatchedMCMC(W, 6, used, [used], 0, pmin, pmax, P0, np.zeros(6), seed_ij=2015, seed_kl=1262)
    s.set_covariance(np.diag(width ** 2))
    th = syn.walker_theory(1, seed=11, lmax=2508, n_fields=6)
    s.add_likelihood(like, torch.tensor(th, device="cuda").expand(W, 6, th.shape[2]))
    g = syn.gaussians(17, W * 6).reshape(W, 6)
    s.set_start(P0[None, :] + g * width[None, :])
    s.enable_history(steps)
    s.step(steps, fast_only=True)
    P, lk, mult, nacc = s.state()
    assert nacc.sum() > W                    # the chains moved
    o = co.CMBLikesOracle(smica_data["gaussian"], over, "SMICA")
    for w in (0, W // 2, W - 1):
        assert lk[w] == pytest.approx(o.loglike(th[0], P[w]), rel=1e-10)
    der = LikelihoodDerived(ll, used, P0)
    assert der.names == [("Dl2000_smica", "Dl2000_smica")]
    rows = s.history_host(0, steps)          # [steps, n_used + 1, W]
    cols = der.columns(rows[:, :6, :])
    for t in (0, steps - 1):
        for w in (0, W - 1):
            assert cols[t, 0, w] == pytest.approx(o.derived(rows[t, :6, w])[0], rel=1e-13)
    root = str(tmp_path / "smica_chain")
    cw = ChainWriter(root, names, likelihoods=[like.description()], derived=der, burn_in=0)
    cw.append(s)
    cw.close()
    pn = open(root + ".paramnames").read().split("\n")
    assert pn[6].startswith("Dl2000_smica*") and pn[7].startswith("chi2_SMICA*")
    data = np.loadtxt(root + "_1.txt", ndmin=2)
    assert data.shape[1] == 1 + 1 + 6 + 1 + 2
    np.testing.assert_allclose(data[:, 8], data[:, 2] + data[:, 5], rtol=2e-6)   # A1 + A2 at l = pivot
    s.close()
