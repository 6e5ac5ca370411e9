"""The C restatement (oracle/liboracle.so) against the compiled reference.

Fixtures in tests/golden/ were produced by oracle/gen_golden.py from the
reference's own Fortran (built from /root/reference by oracle/Makefile).
CPU only.
"""
import numpy as np
import pytest

import pyoracle as po
from cosmomc_amd import synthetic as syn

PLIK_SEL = {"plik_lite_TTTEEE": ("TT TE EE", None), "plik_lite_TT": ("TT", None),
            "plik_lite_TE": ("TE", None), "plik_lite_TTEE": ("TT EE", None),
            "plik_lite_TTTEEE_Lrange": ("TT TE EE", (100, 1500))}


def test_ranmar_known_answer(rng_golden):
    # RandUtils.f90:262-283 (Marsaglia-Zaman-James test values)
    expect = [6533892.0, 14220222.0, 7275067.0, 6172232.0, 8354498.0, 10633180.0]
    assert rng_golden["kat"] == expect
    r = po.Ranmar(1802, 9373)
    r.ranmar(20000)
    assert list(r.ranmar(6) * 4096.0 * 4096.0) == expect


@pytest.mark.parametrize("key", ["1802_9373", "1234_5678", "31328_30081"])
def test_rng_streams_bitexact(rng_golden, key):
    g = rng_golden["streams"][key]
    n = len(g["ranmar"])
    r = po.Ranmar(g["ij"], g["kl"])
    assert np.array_equal(r.ranmar(n), np.array(g["ranmar"]))              # bit-exact
    gs = np.array([r.gaussian1() for _ in range(n)])
    np.testing.assert_allclose(gs, g["gaussian1"], rtol=2e-15, atol=0)
    ex = np.array([r.randexp1() for _ in range(n)], dtype=np.float64)
    assert np.array_equal(ex.astype(np.float32), np.array(g["randexp1"]).astype(np.float32))
    assert list(r.rand_indices(g["nidx"], g["nidx"])) == g["rand_indices"]
    R = r.rand_rotation(g["nrot"])
    np.testing.assert_allclose(R.ravel(), g["rotation"], rtol=0, atol=1e-14)


@pytest.mark.parametrize("case", list(PLIK_SEL))
def test_oracle_plik_lite_vs_reference(plik_golden, case):
    g = plik_golden
    c = g["cases"][case]
    data = syn.make_plik_lite(g["data_seed"])
    use, rng = PLIK_SEL[case]
    P = po.PlikLite(data, use, rng)
    th = syn.walker_theory(c["walkers"], seed=g["theory_seed"], n_fields=3)
    got = P.loglike_batch(th, np.array(c["cal"]))
    np.testing.assert_allclose(got, c["minus_lnL"], rtol=1e-12, atol=0)


def _target(ch):
    """orc_target_t of a golden chain: test Gaussian over params_used, bounds,
    Gaussian priors (varying / include_fixed gate) and linear-combination priors."""
    n = ch["n"]
    npar = ch.get("num_params", n)
    used = np.array(ch.get("params_used", list(range(1, n + 1))), dtype=np.int32)
    keep = {k: np.ascontiguousarray(ch[k], dtype=np.float64) for k in
            ("pmin", "pmax", "prior_mean", "prior_std", "center")}
    covinv = np.ascontiguousarray(np.array(ch["cov"], dtype=np.float64))
    assert po.lib().orc_matrix_inverse(covinv, n) == 0
    keep["covinv"] = covinv
    keep["used"] = used
    vary = np.zeros(npar, dtype=np.int32)
    vary[used - 1] = 1
    keep["vary"] = vary
    lin = ch.get("linear_combinations", [])
    keep["lw"] = np.ascontiguousarray([lc["weights"] for lc in lin] or [[0.0]], dtype=np.float64)
    keep["lm"] = np.ascontiguousarray([lc["mean"] for lc in lin] or [0.0], dtype=np.float64)
    keep["ls"] = np.ascontiguousarray([lc["std"] for lc in lin] or [0.0], dtype=np.float64)
    t = po.Target()
    t.num_params = npar
    t.pmin, t.pmax = keep["pmin"].ctypes.data, keep["pmax"].ctypes.data
    t.prior_mean, t.prior_std = keep["prior_mean"].ctypes.data, keep["prior_std"].ctypes.data
    t.temperature = ch["temperature"]
    t.test_like, t.n_used = 1, n
    t.params_used = keep["used"].ctypes.data
    t.test_covinv, t.center = keep["covinv"].ctypes.data, keep["center"].ctypes.data
    t.include_fixed_parameter_priors = int(ch.get("include_fixed_parameter_priors", 0))
    t.varying = keep["vary"].ctypes.data
    t.n_lincomb = len(lin)
    t.lincomb_weights, t.lincomb_mean, t.lincomb_std = (keep["lw"].ctypes.data, keep["lm"].ctypes.data,
                                                        keep["ls"].ctypes.data)
    return t, keep


def make_oracle_proposer(ch):
    blocks = ch["blocks"]
    bn = np.array([len(b) for b in blocks], dtype=np.int32)
    bp = np.array([x for b in blocks for x in b], dtype=np.int32)
    pu = np.array(ch.get("params_used", list(range(1, ch["n"] + 1))), dtype=np.int32)
    h = po.lib().orc_proposer_create(len(blocks), bn, bp, ch["slow_block_max"], ch["oversample_fast"],
                                     ch["propose_scale"], ch["n"], pu)
    po.lib().orc_proposer_set_covariance(h, np.ascontiguousarray(ch["cov"], dtype=np.float64))
    return h


MH_CHAINS = ["gauss6_single_block", "gauss6_blocked", "gauss6_fast_only", "gauss3_n1_blocks",
             "gauss27_fast21_fast_only", "gauss27_fast21_os3", "gauss27_fast12_9_lincomb", "gauss40_slow_fast"]
DRAG_CHAINS = ["gauss6_drag", "gauss4_drag_every_step", "gauss27_fast21_drag"]


@pytest.mark.parametrize("name", MH_CHAINS)
def test_oracle_chain_vs_reference(rng_golden, name):
    import ctypes as C
    ch = rng_golden["chains"][name]
    t, keep = _target(ch)
    h = make_oracle_proposer(ch)
    r = po.Ranmar(ch["ij"], ch["kl"])
    P = np.array(ch["P0"], dtype=np.float64)
    cur = C.c_double(po.lib().orc_target_loglike(C.byref(t), P))
    assert cur.value == pytest.approx(ch["like0"], rel=1e-13)
    tl = C.c_double(0.0)
    for k in range(ch["steps"]):
        acc = po.lib().orc_mh_step(h, C.byref(r.s), C.byref(t), P, C.byref(cur), ch["fast_only"], C.byref(tl))
        assert acc == ch["accept"][k], f"accept mismatch at step {k}"
        i = ch["at"][k]
        if i is not None:
            assert tl.value == pytest.approx(ch["trial_like"][i], rel=1e-10, abs=1e-12)
            assert cur.value == pytest.approx(ch["cur_like"][i], rel=1e-10, abs=1e-12)
            np.testing.assert_allclose(P, ch["P"][i], rtol=1e-11, atol=1e-12)
    po.lib().orc_proposer_free(h)


def test_gelman_rubin_identity():
    # equal within-chain covariances and zero spread of means -> R-1 = 0
    n = 4
    cov = np.diag([1.0, 2.0, 3.0, 4.0])
    assert po.lib().orc_gelman_rubin(cov, np.zeros((n, n)), n) == pytest.approx(0.0, abs=1e-15)
    # between-chain covariance equal to within -> largest eigenvalue 1
    assert po.lib().orc_gelman_rubin(cov, cov.copy(), n) == pytest.approx(1.0, rel=1e-12)


@pytest.mark.parametrize("name", DRAG_CHAINS)
def test_oracle_dragging_vs_reference(rng_golden, name):
    """TFastDraggingSampler_GetNewSample (MCMC.f90:338-452) step by step."""
    import ctypes as C
    ch = rng_golden["chains"][name]
    t, keep = _target(ch)
    h = make_oracle_proposer(ch)
    r = po.Ranmar(ch["ij"], ch["kl"])
    P = np.array(ch["P0"], dtype=np.float64)
    cur = C.c_double(po.lib().orc_target_loglike(C.byref(t), P))
    st = po.DragState(0, 1.0, 3.0, ch["oversample_fast"])
    for k in range(ch["steps"]):
        acc = po.lib().orc_drag_step(h, C.byref(r.s), C.byref(t), C.byref(st), P, C.byref(cur))
        assert acc == ch["accept"][k], f"accept mismatch at step {k}"
        i = ch["at"][k]
        if i is not None:
            assert cur.value == pytest.approx(ch["cur_like"][i], rel=1e-10, abs=1e-12)
            np.testing.assert_allclose(P, ch["P"][i], rtol=1e-11, atol=1e-12)
    po.lib().orc_proposer_free(h)
