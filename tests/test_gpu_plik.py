"""plik_lite HIP kernels vs the compiled reference (golden fixtures) and the
C restatement (oracle/liboracle.so).  GPU only.

Tolerances: fp64 throughout; the GPU sums the quadratic form in a different
order (MFMA blocks, symmetric upper-block triangle) than DSYMV, so results
agree to rounding: rtol 1e-10 on -lnL (north star: |d lnL| < 1e-6).
"""
import numpy as np
import pytest

import pyoracle as po
from cosmomc_amd import synthetic as syn

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

RTOL = 1e-10

CASES = {"plik_lite_TTTEEE": {}, "plik_lite_TT": {"use_cl": "TT"}, "plik_lite_TE": {"use_cl": "TE"},
         "plik_lite_TTEE": {"use_cl": "TT EE"}, "plik_lite_TTTEEE_Lrange": {"bins_for_L_range": "100 1500"}}
ORACLE_SEL = {"plik_lite_TTTEEE": ("TT TE EE", None), "plik_lite_TT": ("TT", None),
              "plik_lite_TE": ("TE", None), "plik_lite_TTEE": ("TT EE", None),
              "plik_lite_TTTEEE_Lrange": ("TT TE EE", (100, 1500))}


@pytest.fixture(scope="module")
def data():
    return syn.make_plik_lite(12345)


@pytest.fixture(scope="module")
def dataset(tmp_path_factory, data):
    return data.write(str(tmp_path_factory.mktemp("plik")))


def _open(dataset, over=None):
    from cosmomc_amd.likelihood import NativeCMBLikelihood
    return NativeCMBLikelihood("PLIK_LITE", dataset, over or {})


def test_native_library_is_the_path():
    from cosmomc_amd import _native as N
    assert torch.cuda.is_available()
    N.lib()  # loads cosmomc_amd/lib/libcosmomc_amd.so


@pytest.mark.parametrize("case", list(CASES))
def test_plik_vs_reference_golden(plik_golden, dataset, case):
    c = plik_golden["cases"][case]
    like = _open(dataset, CASES[case])
    assert like.nuisance_names == ["calPlanck"]
    th = torch.tensor(syn.walker_theory(c["walkers"], seed=plik_golden["theory_seed"], n_fields=3), device="cuda")
    cal = torch.tensor(c["cal"], dtype=torch.float64, device="cuda").reshape(-1, 1)
    got = like.loglike_batch(th, cal).cpu().numpy()
    np.testing.assert_allclose(got, c["minus_lnL"], rtol=RTOL, atol=0)


@pytest.mark.parametrize("W", [1, 2, 63, 64, 65, 130, 257])
def test_plik_walker_counts_vs_oracle(data, dataset, W):
    like = _open(dataset)
    orc = po.PlikLite(data)
    th = syn.walker_theory(W, seed=777, n_fields=3)
    cal = syn.walker_calibrations(W, seed=99)
    got = like.loglike_batch(torch.tensor(th, device="cuda"), torch.tensor(cal, device="cuda").reshape(-1, 1))
    ref = orc.loglike_batch(th, cal)
    np.testing.assert_allclose(got.cpu().numpy(), ref, rtol=RTOL, atol=0)


def test_plik_strided_layouts(data, dataset):
    """ld_field / ld_walker larger than the data (padded rows, 10-field layout)."""
    like = _open(dataset)
    orc = po.PlikLite(data)
    W = 37
    th = syn.walker_theory(W, seed=5, n_fields=3)
    big = np.zeros((W, 10, 2600))
    big[:, :3, :2509] = th
    cal = syn.walker_calibrations(W, seed=6)
    nu = np.zeros((W, 3))
    nu[:, 1] = cal                      # nuisance taken from a strided column view
    tb = torch.tensor(big, device="cuda")
    tn = torch.tensor(nu, device="cuda")[:, 1:2]
    got = like.loglike_batch(tb, tn).cpu().numpy()
    np.testing.assert_allclose(got, orc.loglike_batch(th, cal), rtol=RTOL, atol=0)


def test_plik_host_entry(data, dataset):
    like = _open(dataset)
    orc = po.PlikLite(data)
    th = syn.walker_theory(9, seed=8, n_fields=3)
    cal = syn.walker_calibrations(9, seed=9)
    np.testing.assert_allclose(like.loglike_host(th, cal[:, None]), orc.loglike_batch(th, cal), rtol=RTOL)


def test_plik_host_entry_per_eval_loop(data, dataset):
    """The Fortran LogLike binding calls the host entry once per evaluation
    (W = 1): buffers persist on the handle, so a call costs tens of
    microseconds, not allocations; a shared theory (ld_walker = 0) reads only
    the fields the likelihood uses."""
    import ctypes as C
    import time
    from cosmomc_amd import _native as N
    like = _open(dataset)
    orc = po.PlikLite(data)
    th = syn.walker_theory(40, seed=18, n_fields=3)
    cal = syn.walker_calibrations(40, seed=19)
    like.loglike_host(th[:1], cal[:1, None])                  # sizes the staging once
    t0 = time.perf_counter()
    got = np.array([like.loglike_host(th[w:w + 1], cal[w:w + 1, None])[0] for w in range(40)])
    per_call = (time.perf_counter() - t0) / 40
    np.testing.assert_allclose(got, orc.loglike_batch(th, cal), rtol=RTOL)
    print(f"host entry W=1: {per_call * 1e6:.1f} us per call")
    assert per_call < 1e-3
    one = np.ascontiguousarray(th[3])                          # [3, L]: exactly the fields plik_lite reads
    W = 7
    out = np.empty(W)
    nu = np.ascontiguousarray(cal[:W, None])
    rc = N.lib().cmbl_loglike_batch_host(like._h, W, one.ctypes.data, one.shape[1], 0, nu.ctypes.data, 1,
                                         out.ctypes.data)
    N.check(rc, like._h)
    np.testing.assert_allclose(out, [orc.loglike(one, c) for c in cal[:W]], rtol=RTOL)


def test_plik_zero_theory_property(data, dataset):
    """Zero theory: every walker's -lnL is X^T C^-1 X / 2, independent of cal."""
    like = _open(dataset)
    W = 300
    th = torch.zeros((W, 3, 2509), dtype=torch.float64, device="cuda")
    cal = torch.linspace(0.95, 1.05, W, dtype=torch.float64, device="cuda").reshape(-1, 1)
    got = like.loglike_batch(th, cal).cpu().numpy()
    ref = po.PlikLite(data).loglike(np.zeros((3, 2509)), 1.0)
    np.testing.assert_allclose(got, np.full(W, ref), rtol=RTOL)


def test_plik_full_size_sampled(data, dataset):
    """BASELINE size W=4096: spot-check 64 walkers against the oracle and the
    cal-scaling identity -lnL(D, cal) == -lnL(D / cal^2, 1) for all walkers."""
    like = _open(dataset)
    W = 4096
    th = torch.tensor(syn.walker_theory(W, seed=31, n_fields=3), device="cuda")
    cal = torch.tensor(syn.walker_calibrations(W, seed=32), device="cuda").reshape(-1, 1)
    a = like.loglike_batch(th, cal)
    b = like.loglike_batch(th / (cal * cal).reshape(-1, 1, 1), torch.ones_like(cal))
    np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), rtol=1e-9)
    idx = np.arange(0, W, 64)
    orc = po.PlikLite(data)
    ref = orc.loglike_batch(th[idx].cpu().numpy(), cal[idx, 0].cpu().numpy())
    np.testing.assert_allclose(a[idx].cpu().numpy(), ref, rtol=RTOL)


def test_clik_packing_routes_to_native(data, dataset):
    """cliklike.f90:138-166 packing: C_l = D_l 2pi/(l(l+1)) for TT EE BB TE (+TB EB = 0)
    followed by the nuisance parameters; clik returns +lnL."""
    from cosmomc_amd.likelihood import ClikLikelihood
    like = ClikLikelihood("PLIK_LITE", dataset)
    W = 5
    th = syn.walker_theory(W, seed=11, n_fields=3)
    cal = syn.walker_calibrations(W, seed=12)
    lmax = [2508, 2508, -1, 2508, -1, -1]          # TT EE BB TE TB EB
    ell = np.arange(2509, dtype=np.float64)
    fac = np.zeros_like(ell)
    fac[2:] = 2 * np.pi / (ell[2:] * (ell[2:] + 1))
    rows = []
    for w in range(W):
        tt, te, ee = th[w, 0] * fac, th[w, 1] * fac, th[w, 2] * fac
        rows.append(np.concatenate([tt, ee, te, [cal[w]]]))
    v = torch.tensor(np.array(rows), device="cuda")
    got = like.clik_compute(v, lmax).cpu().numpy()
    ref = -po.PlikLite(data).loglike_batch(th, cal)
    np.testing.assert_allclose(got, ref, rtol=1e-9)
    ws = like.clik_workspace(W)                   # caller's workspace, on a side stream, no host sync
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        got2 = like.clik_compute(v, lmax, workspace=ws)
    s.synchronize()
    np.testing.assert_allclose(got2.cpu().numpy(), ref, rtol=1e-9)


def test_bad_dataset_errors(tmp_path, dataset):
    from cosmomc_amd import _native as N
    from cosmomc_amd.likelihood import NativeCMBLikelihood
    with pytest.raises(N.NativeError):
        NativeCMBLikelihood("PLIK_LITE", str(tmp_path / "missing.dataset"))
    with pytest.raises(N.NativeError):
        NativeCMBLikelihood("PLIK_LITE", dataset, {"use_cl": "BB"})   # selects no bins
    with pytest.raises(N.NativeError):
        NativeCMBLikelihood("NOT_A_TAG", dataset)


def test_plik_tt_configs1_shape_vs_oracle(data, dataset):
    """BASELINE configs[1]'s shape: plik_lite TT (batch2/plik_lite_TT.ini) on
    one fixed theory (the reference's base_plikHM best fit, ld_walker = 0) for
    256 walkers with their own calibrations: every walker's -lnL equals the
    C oracle's (TT selection) to rtol 1e-10."""
    like = _open(dataset, {"use_cl": "TT"})
    orc = po.PlikLite(data, "TT")
    W = 256
    base = syn.base_theory()[:3]
    th = torch.tensor(base, device="cuda").reshape(1, 3, -1).expand(W, 3, base.shape[-1])
    cal = syn.walker_calibrations(W, seed=256)
    got = like.loglike_batch(th, torch.tensor(cal, device="cuda").reshape(-1, 1)).cpu().numpy()
    ref = np.array([orc.loglike(base, c) for c in cal])
    np.testing.assert_allclose(got, ref, rtol=RTOL, atol=0)
