"""Batched Metropolis / BlockedProposer on the GPU vs the reference chains
(golden fixtures from the compiled Fortran) and the C restatement.  GPU only.

Walker 0 is seeded with the reference chain's (ij, kl), so its whole
trajectory must follow the reference chain: identical accept/reject
decisions, parameters to rounding (the GPU's log/sqrt may differ from libm by
an ulp, hence rtol 1e-11 rather than bit equality).
"""
import ctypes as C

import numpy as np
import pytest

import pyoracle as po
from cosmomc_amd import synthetic as syn

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

CHAINS = ["gauss6_single_block", "gauss6_blocked", "gauss6_fast_only", "gauss3_n1_blocks"]
# BASELINE configs[3] shapes: 21-parameter fast blocks (rotations read in place from HBM when the
# LDS image is full), a 12 + 9 split, 40 used parameters, fixed parameters and linear-combination priors
WIDE_CHAINS = ["gauss27_fast21_fast_only", "gauss27_fast21_os3", "gauss27_fast12_9_lincomb", "gauss40_slow_fast"]


def _make_sampler(ch, W):
    from cosmomc_amd.sampler import BatchedMCMC
    n = ch["n"]
    npar = ch.get("num_params", n)
    lin = [(lc["weights"], lc["mean"], lc["std"]) for lc in ch.get("linear_combinations", [])]
    s = BatchedMCMC(W, npar, ch.get("params_used", list(range(1, n + 1))), ch["blocks"], ch["slow_block_max"],
                    ch["pmin"], ch["pmax"], ch["prior_mean"], ch["prior_std"], oversample_fast=ch["oversample_fast"],
                    propose_scale=ch["propose_scale"], temperature=ch["temperature"], seed_ij=ch["ij"],
                    seed_kl=ch["kl"], include_fixed_parameter_priors=bool(ch.get("include_fixed_parameter_priors")),
                    linear_combinations=lin)
    s.set_covariance(np.array(ch["cov"]))
    s.set_test_gaussian(np.array(ch["cov"]), np.array(ch["center"]))
    s.set_start(np.tile(np.array(ch["P0"]), (W, 1)))
    return s


def _oracle_chain(ch, ij, kl, steps):
    from test_oracle import _target, make_oracle_proposer
    t, keep = _target(ch)
    h = make_oracle_proposer(ch)
    r = po.Ranmar(ij, kl)
    P = np.array(ch["P0"], dtype=np.float64)
    cur = C.c_double(po.lib().orc_target_loglike(C.byref(t), P))
    tl = C.c_double(0.0)
    Ps, likes = [], []
    for _ in range(steps):
        po.lib().orc_mh_step(h, C.byref(r.s), C.byref(t), P, C.byref(cur), ch["fast_only"], C.byref(tl))
        Ps.append(P.copy())
        likes.append(cur.value)
    po.lib().orc_proposer_free(h)
    return np.array(Ps), np.array(likes)


@pytest.mark.parametrize("name", CHAINS + WIDE_CHAINS)
def test_walker0_follows_reference_chain(rng_golden, name):
    ch = rng_golden["chains"][name]
    W = 8
    s = _make_sampler(ch, W)
    P, like, mult, nacc = s.state()
    assert like[0] == pytest.approx(ch["like0"], rel=1e-13)
    for k in range(ch["steps"]):
        prev = P[0].copy()
        s.step(1, fast_only=bool(ch["fast_only"]))
        P, like, mult, nacc = s.state()
        assert int(np.any(P[0] != prev)) == ch["accept"][k], f"accept decision at step {k}"
        i = ch["at"][k]
        if i is not None:
            np.testing.assert_allclose(P[0], ch["P"][i], rtol=1e-11, atol=1e-12, err_msg=f"step {k}")
            assert like[0] == pytest.approx(ch["cur_like"][i], rel=1e-10, abs=1e-12)
    assert int(nacc[0]) <= int(sum(ch["accept"]))


@pytest.mark.parametrize("name", ["gauss6_blocked", "gauss3_n1_blocks"])
def test_all_walkers_vs_oracle(rng_golden, name):
    from cosmomc_amd.sampler import walker_seed
    ch = rng_golden["chains"][name]
    W, steps = 70, 150
    s = _make_sampler(ch, W)
    s.step(steps, fast_only=bool(ch["fast_only"]))
    P, like, _, _ = s.state()
    for w in (1, 17, 63, 64, 69):
        ij, kl = walker_seed(ch["ij"], ch["kl"], w)
        Ps, likes = _oracle_chain(ch, ij, kl, steps)
        np.testing.assert_allclose(P[w], Ps[-1], rtol=1e-10, atol=1e-11)
        assert like[w] == pytest.approx(likes[-1], rel=1e-9)


@pytest.mark.parametrize("name", WIDE_CHAINS)
def test_wide_chains_many_walkers_vs_oracle(rng_golden, name):
    """W = 576 (nine 64-walker blocks): walkers 1, 63, 64 and W-1 follow the C
    oracle's chains with their own seeds over every step of the golden run."""
    from cosmomc_amd.sampler import walker_seed
    ch = rng_golden["chains"][name]
    W, steps = 576, ch["steps"]
    s = _make_sampler(ch, W)
    s.step(steps, fast_only=bool(ch["fast_only"]))
    P, like, _, _ = s.state()
    for w in (1, 63, 64, W - 1):
        ij, kl = walker_seed(ch["ij"], ch["kl"], w)
        Ps, likes = _oracle_chain(ch, ij, kl, steps)
        np.testing.assert_allclose(P[w], Ps[-1], rtol=1e-10, atol=1e-11, err_msg=f"walker {w}")
        assert like[w] == pytest.approx(likes[-1], rel=1e-9)


@pytest.mark.parametrize("case", ["TTTEEE_per_walker", "TT_configs1"])
def test_plik_fast_chain_vs_oracle(tmp_path, case):
    """Fast-only Metropolis on calPlanck with native plik_lite + the calPlanck
    prior (batch2/planck_calibration.ini): TTTEEE on per-walker cached theory
    (96 walkers), and BASELINE configs[1]'s shape -- plik_lite TT
    (batch2/plik_lite_TT.ini) on one fixed theory (the reference's
    base_plikHM best fit, ld_walker = 0) for 256 walkers.  The one fast
    parameter takes the lean chain (mhlean.h); checked walkers follow the C
    oracle's chain step by step."""
    from cosmomc_amd.likelihood import NativeCMBLikelihood
    from cosmomc_amd.sampler import BatchedMCMC, walker_seed
    data = syn.make_plik_lite(12345)
    tt = case == "TT_configs1"
    like = NativeCMBLikelihood("PLIK_LITE", data.write(str(tmp_path), use_cl="TT" if tt else "TT TE EE"))
    like.nuisance_indices = [2]
    W, steps = (256, 40) if tt else (96, 60)
    if tt:
        base = syn.base_theory()[:3]
        th = np.broadcast_to(base, (W,) + base.shape)
        dl = torch.tensor(base, device="cuda").reshape(1, 3, -1).expand(W, 3, base.shape[-1])
    else:
        th = syn.walker_theory(W, seed=3, n_fields=3)
        dl = torch.tensor(th, device="cuda")
    np_ = 3
    P0 = np.array([0.0222, 1.0, 3.05])
    pmin = np.array([0.0222, 0.9, 3.05])
    pmax = np.array([0.0222, 1.1, 3.05])
    pm = np.array([0.0, 1.0, 0.0])
    ps = np.array([0.0, 0.0025, 0.0])
    s = BatchedMCMC(W, np_, [2], [[1]], 0, pmin, pmax, pm, ps, propose_scale=2.4, seed_ij=55, seed_kl=66)
    s.set_covariance(np.array([[0.002 ** 2]]))
    s.add_likelihood(like, dl)
    s.set_start(np.tile(P0, (W, 1)))
    s.step(steps, fast_only=True)
    P, lk, _, nacc = s.state()
    assert np.all(nacc > 0)
    orc = po.PlikLite(data, "TT" if tt else "TT TE EE")
    for w in ((0, 127, 128, 255) if tt else (0, 5, 64, 95)):
        ij, kl = walker_seed(55, 66, w)
        bn = np.array([1], dtype=np.int32)
        h = po.lib().orc_proposer_create(1, bn, np.array([1], dtype=np.int32), 0, 1, 2.4, 1,
                                         np.array([2], dtype=np.int32))
        po.lib().orc_proposer_set_covariance(h, np.array([0.002 ** 2]))
        t = po.Target()
        keep = [np.ascontiguousarray(a) for a in (pmin, pmax, pm, ps)]
        dlw = np.ascontiguousarray(th[w])
        t.num_params = np_
        t.pmin, t.pmax, t.prior_mean, t.prior_std = [a.ctypes.data for a in keep]
        t.temperature = 1.0
        t.plik, t.plik_nuis_index, t.plik_dl, t.plik_ld_field = orc.h, 2, dlw.ctypes.data, dlw.shape[1]
        r = po.Ranmar(ij, kl)
        Q = P0.copy()
        cur = C.c_double(po.lib().orc_target_loglike(C.byref(t), Q))
        for _ in range(steps):
            po.lib().orc_mh_step(h, C.byref(r.s), C.byref(t), Q, C.byref(cur), 1, None)
        po.lib().orc_proposer_free(h)
        np.testing.assert_allclose(P[w], Q, rtol=1e-11)
        assert lk[w] == pytest.approx(cur.value, rel=1e-9)


def test_history_stats():
    """Per-walker second-half mean/cov on device == numpy on the same trajectory."""
    from cosmomc_amd.sampler import BatchedMCMC
    n, W = 2, 16
    s = BatchedMCMC(W, n, [1, 2], [[1, 2]], 1, [-10, -10], [10, 10], seed_ij=7, seed_kl=8)
    s.set_covariance(np.eye(2))
    s.set_test_gaussian(np.array([[1.0, 0.3], [0.3, 2.0]]), np.zeros(2))
    s.set_start(np.zeros((W, n)))
    s.enable_history(64)
    traj = []
    for _ in range(40):
        s.step(1)
        traj.append(s.state()[0].copy())
    traj = np.array(traj)                 # [40, W, n]
    m, c = s.history_stats(20, 39)
    x = traj[20:40]
    mu = x.mean(axis=0)
    d = x - mu
    cov = np.einsum("twi,twj->wij", d, d) / x.shape[0]
    np.testing.assert_allclose(m.cpu().numpy(), mu, rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(c.cpu().numpy(), cov, rtol=1e-10, atol=1e-13)


@pytest.mark.parametrize("n", [5, 12, 21, 40])
def test_history_stats_wide(n):
    """hist_mean_kernel / hist_cov_kernel at every register width (8, 16, 32,
    64 parameters), over a wrapped ring and a walker count that is not a
    multiple of 64, against numpy on history_host's rows."""
    from cosmomc_amd.sampler import BatchedMCMC
    W, cap, steps = 100, 48, 70
    used = list(range(1, n + 1))
    rng = np.random.default_rng(n)
    A = rng.standard_normal((n, n))
    cov = A @ A.T / n + np.eye(n)
    s = BatchedMCMC(W, n, used, [used[:n // 2], used[n // 2:]], 1, -50 * np.ones(n), 50 * np.ones(n),
                    seed_ij=11, seed_kl=12)
    s.set_covariance(np.eye(n) * 0.3)
    if n <= 32:      # a 40-d test Gaussian's tables do not fit the LDS image: flat target in the box
        s.set_test_gaussian(cov, np.zeros(n))
    s.set_start(rng.standard_normal((W, n)))
    s.enable_history(cap)
    s.step(steps)
    first, last = steps - 40, steps - 1
    rows = s.history_host(first, last - first + 1)          # [T, n + 1, W]
    x = np.transpose(rows[:, :n, :], (0, 2, 1))             # [T, W, n]
    mu = x.mean(axis=0)
    d = x - mu
    ref = np.einsum("twi,twj->wij", d, d) / x.shape[0]
    m, c = s.history_stats(first, last)
    np.testing.assert_allclose(m.cpu().numpy(), mu, rtol=1e-12, atol=1e-13)
    np.testing.assert_allclose(c.cpu().numpy(), ref, rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("groups", [2, 3, 8])
def test_walker_groups_same_chains(tmp_path, groups):
    """cmbs_set_groups only changes how the step is scheduled: every walker's
    chain is the one the single-stream path produces (the quadratic-form
    split may differ with the group size, so -lnL agrees to rounding and the
    accept decisions exactly)."""
    from cosmomc_amd.likelihood import NativeCMBLikelihood
    from cosmomc_amd.sampler import BatchedMCMC
    data = syn.make_plik_lite(12345)
    like = NativeCMBLikelihood("PLIK_LITE", data.write(str(tmp_path)))
    like.nuisance_indices = [2]
    W, steps = 200, 25
    dl = torch.tensor(syn.walker_theory(W, seed=4, n_fields=3), device="cuda")
    P0 = np.array([0.0222, 1.0])
    pmin, pmax = np.array([0.0222, 0.9]), np.array([0.0222, 1.1])
    pm, ps = np.array([0.0, 1.0]), np.array([0.0, 0.0025])
    runs = []
    for g in (1, groups):
        s = BatchedMCMC(W, 2, [2], [[1]], 0, pmin, pmax, pm, ps, propose_scale=2.4, seed_ij=3, seed_kl=4)
        s.set_covariance(np.array([[0.002 ** 2]]))
        s.set_groups(g)
        s.add_likelihood(like, dl)
        s.set_start(np.tile(P0, (W, 1)))
        s.enable_history(steps)
        s.step(steps, fast_only=True)
        P, lk, mult, nacc = s.state()
        m, _ = s.history_stats(0, steps - 1)
        runs.append((P.copy(), lk.copy(), mult.copy(), nacc.copy(), m.cpu().numpy()))
        s.close()
    a, b = runs
    np.testing.assert_array_equal(a[3], b[3])
    np.testing.assert_array_equal(a[2], b[2])
    np.testing.assert_allclose(b[0], a[0], rtol=1e-12)
    np.testing.assert_allclose(b[1], a[1], rtol=1e-10)
    np.testing.assert_allclose(b[4], a[4], rtol=1e-12)


def test_convergence_exchange_on_device():
    """cmbs_chain_moments + ConvergenceExchange (world 1) == the reference
    pooling restated in the oracle over the same per-walker trajectories."""
    from cosmomc_amd.converge import CollectorSettings, ConvergenceExchange, reference_window
    from cosmomc_amd.sampler import BatchedMCMC
    n, W, T = 3, 70, 60
    s = BatchedMCMC(W, n, [1, 2, 3], [[1, 2], [3]], 1, [-10] * 3, [10] * 3, seed_ij=17, seed_kl=18)
    cov = np.array([[1.0, 0.3, 0.1], [0.3, 2.0, 0.2], [0.1, 0.2, 0.5]])
    s.set_covariance(cov)
    s.set_test_gaussian(cov, np.zeros(n))
    s.set_start(np.tile([0.5, -0.5, 0.2], (W, 1)))
    s.enable_history(T)
    traj = []
    for _ in range(T):
        s.step(1)
        traj.append(s.state()[0].copy())
    traj = np.array(traj).transpose(1, 0, 2)          # [W, T, n]
    ref = po.pool_chain_statistics(list(traj))
    first, last = reference_window(T)
    ex = ConvergenceExchange(n, CollectorSettings(MPI_Min_Sample_Update=20))
    r = ex.update_cov_and_check_converge(s, first, last)
    np.testing.assert_allclose(r.mean, ref["mean"], rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(r.propose_cov, ref["propose_cov"], rtol=1e-10, atol=1e-14)
    np.testing.assert_allclose(r.cov, ref["cov"], rtol=1e-10, atol=1e-14)
    np.testing.assert_allclose(r.meanscov, ref["meanscov"], rtol=1e-8, atol=1e-14)
    assert r.R == pytest.approx(po.gelman_rubin(ref["cov"], ref["meanscov"]), rel=1e-8)
    s.set_covariance(r.propose_cov)                   # learnt proposal (SetCovariance, :317)
    s.step(5)
    assert np.all(np.isfinite(s.state()[1]))


@pytest.mark.parametrize("name", ["gauss6_drag", "gauss4_drag_every_step", "gauss27_fast21_drag"])
def test_walker0_follows_reference_dragging(rng_golden, name):
    """cmbs_step_drag: walker 0 (seeded as the reference chain) follows the
    reference TFastDraggingSampler chain step by step; every walker follows
    the C oracle's dragging chain with its own seed."""
    from cosmomc_amd.sampler import walker_seed
    from test_oracle import _target, make_oracle_proposer
    ch = rng_golden["chains"][name]
    W = 70
    s = _make_sampler(ch, W)
    P = s.state()[0]
    for k in range(ch["steps"]):
        prev = P[0].copy()
        s.step_drag(1)
        P, like, mult, nacc = s.state()
        assert int(np.any(P[0] != prev)) == ch["accept"][k], f"accept decision at step {k}"
        i = ch["at"][k]
        if i is not None:
            np.testing.assert_allclose(P[0], ch["P"][i], rtol=1e-11, atol=1e-12, err_msg=f"step {k}")
            assert like[0] == pytest.approx(ch["cur_like"][i], rel=1e-10, abs=1e-12)
    t, keep = _target(ch)
    for w in (1, 37, 69):
        ij, kl = walker_seed(ch["ij"], ch["kl"], w)
        h = make_oracle_proposer(ch)
        r = po.Ranmar(ij, kl)
        Q = np.array(ch["P0"], dtype=np.float64)
        cur = C.c_double(po.lib().orc_target_loglike(C.byref(t), Q))
        st = po.DragState(0, 0.0, 3.0, ch["oversample_fast"])   # SampleFrom starts with mult = 0 (MCMC.f90:141)
        for _ in range(ch["steps"]):
            po.lib().orc_drag_step(h, C.byref(r.s), C.byref(t), C.byref(st), Q, C.byref(cur))
        po.lib().orc_proposer_free(h)
        np.testing.assert_allclose(P[w], Q, rtol=1e-10, atol=1e-12)
        assert mult[w] == st.mult


def test_dragging_with_plik_theory_callback(tmp_path):
    """Dragging over a slow amplitude A (theory = A x base D_l, supplied by a
    theory function at every drag) with calPlanck fast and plik_lite: after the
    run every walker's theory row is A_w x base (accepted drags swapped it in)
    and its CurLike is the oracle's -lnL there plus the calPlanck prior."""
    from cosmomc_amd.likelihood import NativeCMBLikelihood
    from cosmomc_amd.sampler import BatchedMCMC
    data = syn.make_plik_lite(12345)
    like = NativeCMBLikelihood("PLIK_LITE", data.write(str(tmp_path)))
    like.nuisance_indices = [2]
    W = 64
    base = torch.tensor(syn.base_theory(2508)[:3], device="cuda")
    theory = base.unsqueeze(0).repeat(W, 1, 1).contiguous()
    end = torch.empty_like(theory)
    pmin, pmax = np.array([0.9, 0.9]), np.array([1.1, 1.1])
    pm, ps = np.array([0.0, 1.0]), np.array([0.0, 0.0025])
    s = BatchedMCMC(W, 2, [1, 2], [[1], [2]], 1, pmin, pmax, pm, ps, oversample_fast=2, propose_scale=2.4,
                    seed_ij=91, seed_kl=92)
    s.set_covariance(np.diag([0.003 ** 2, 0.0025 ** 2]))
    s.add_likelihood(like, theory)
    s.set_drag_theory(0, end)
    s.set_start(np.tile([1.0, 1.0], (W, 1)))
    s.enable_history(64)

    def theory_fn(P_end):
        end.copy_(base.unsqueeze(0) * P_end[0].reshape(-1, 1, 1))
    s.step_drag(40, theory_fn=theory_fn)
    P, lk, mult, nacc = s.state()
    terms = s.history_terms(s.history_count() - 1, 1)[0, 0]     # plik -lnL at the current points
    assert np.any(np.abs(P[:, 0] - 1.0) > 1e-6), "no drag was accepted"
    th = theory.cpu().numpy()
    b = base.cpu().numpy()
    orc = po.PlikLite(data)
    for w in range(0, W, 9):
        np.testing.assert_allclose(th[w], P[w, 0] * b, rtol=1e-15, atol=0)
        ref = orc.loglike(th[w], P[w, 1]) + 0.5 * ((P[w, 1] - 1.0) / 0.0025) ** 2
        assert lk[w] == pytest.approx(ref, rel=1e-9)
        assert terms[w] == pytest.approx(orc.loglike(th[w], P[w, 1]), rel=1e-9)


def test_history_terms_and_chi2_chain_files(tmp_path):
    """Per-likelihood terms of the recorded points (cmbs_history_terms_host)
    equal the oracle's plik_lite -lnL at every recorded point, and the chain
    files' chi2_plik / chi2_prior columns follow from them."""
    from cosmomc_amd.chains import ChainWriter
    from cosmomc_amd.likelihood import NativeCMBLikelihood
    from cosmomc_amd.sampler import BatchedMCMC
    data = syn.make_plik_lite(12345)
    like = NativeCMBLikelihood("PLIK_LITE", data.write(str(tmp_path)))
    like.nuisance_indices = [2]
    W, steps = 64, 40
    th = syn.walker_theory(W, seed=3, n_fields=3)
    dl = torch.tensor(th, device="cuda")
    s = BatchedMCMC(W, 3, [2], [[1]], 0, [0.0222, 0.9, 3.05], [0.0222, 1.1, 3.05], [0.0, 1.0, 0.0],
                    [0.0, 0.0025, 0.0], seed_ij=55, seed_kl=66)
    s.set_covariance(np.array([[0.002 ** 2]]))
    s.add_likelihood(like, dl)
    s.enable_history(steps)
    s.set_start(np.tile([0.0222, 1.0, 3.05], (W, 1)))
    cw = ChainWriter(str(tmp_path / "run"), ["calPlanck"], likelihoods=[like.description()], burn_in=-1)
    s.step(steps, fast_only=True)
    cw.append(s)
    open_runs = {w: c[1] for w, c in cw.pending.items()}
    cw.close()
    hist = s.history_host(0, steps)
    terms = s.history_terms(0, steps)
    orc = po.PlikLite(data)
    for w in (0, 17, 63):
        for k in (0, 11, steps - 1):
            cal = hist[k, 0, w]
            assert terms[k, 0, w] == pytest.approx(orc.loglike(th[w], cal), rel=1e-9)
            assert hist[k, 1, w] == pytest.approx(terms[k, 0, w] + 0.5 * ((cal - 1.0) / 0.0025) ** 2, rel=1e-12)
        c = np.loadtxt(tmp_path / f"run_{w + 1}.txt", ndmin=2)
        assert c[:, 0].sum() + open_runs[w] == steps, (w, c[:, :3], hist[:, 0, w])
        # chi2_prior; the file holds calPlanck to 7 digits (1e-6), so compare to 1e-3
        np.testing.assert_allclose(c[:, 4], ((c[:, 2] - 1.0) / 0.0025) ** 2, rtol=0, atol=1e-3)
        np.testing.assert_allclose(c[:, 3] / 2 + c[:, 4] / 2, c[:, 1], rtol=1e-6)                 # chi2s add up
    assert open(tmp_path / "run.likelihoods").read().split("\t")[:3] == ["1", "CMB", "PLIK_LITE"]


@pytest.mark.gpu
def test_deferred_combine_bitwise(tmp_path):
    """In fast steps the plik quadratic form leaves its split-K partials to the
    accepting mh_kernel (QFDeferred); the terms it finishes are bit-identical
    to cmbl_loglike_batch's in-launch combine at the same points (W = 512:
    eight walker tiles, XCD-aware item placement)."""
    from cosmomc_amd.likelihood import NativeCMBLikelihood
    from cosmomc_amd.sampler import BatchedMCMC
    data = syn.make_plik_lite(12345)
    like = NativeCMBLikelihood("PLIK_LITE", data.write(str(tmp_path)))
    like.nuisance_indices = [2]
    W, steps = 512, 12
    th = syn.walker_theory(W, seed=5, n_fields=3)
    dl = torch.tensor(th, device="cuda")
    s = BatchedMCMC(W, 3, [2], [[1]], 0, [0.0222, 0.9, 3.05], [0.0222, 1.1, 3.05], [0.0, 1.0, 0.0],
                    [0.0, 0.0025, 0.0], seed_ij=57, seed_kl=68)
    s.set_covariance(np.array([[0.002 ** 2]]))
    s.add_likelihood(like, dl)
    s.enable_history(steps)
    s.set_start(np.tile([0.0222, 1.0, 3.05], (W, 1)))
    s.step(steps, fast_only=True)
    hist = s.history_host(0, steps)
    terms = s.history_terms(0, steps)
    for k in (0, steps // 2, steps - 1):
        cal = torch.tensor(hist[k, 0, :].copy(), device="cuda").reshape(-1, 1)
        ref = like.loglike_batch(dl, cal).cpu().numpy()
        assert np.array_equal(terms[k, 0], ref), np.abs(terms[k, 0] - ref).max()


@pytest.mark.parametrize("oversample", [1, 3])
def test_full_steps_with_theory_callback(tmp_path, oversample):
    """cmbs_step_theory: full GetNewSample steps (slow amplitude A and fast
    calPlanck) with the theory A x base recomputed at every trial point by a
    theory function.  Walkers follow the C oracle's chains (its slow-theory
    model scales the cached theory by P(A)) and accepted walkers carry A x base."""
    from cosmomc_amd.likelihood import NativeCMBLikelihood
    from cosmomc_amd.sampler import BatchedMCMC, walker_seed
    from cosmomc_amd._native import NativeError
    data = syn.make_plik_lite(12345)
    like = NativeCMBLikelihood("PLIK_LITE", data.write(str(tmp_path)))
    like.nuisance_indices = [2]
    W, steps = 80, 40
    base = torch.tensor(syn.base_theory(2508)[:3], device="cuda")
    theory = base.unsqueeze(0).repeat(W, 1, 1).contiguous()
    trial = torch.empty_like(theory)
    pmin, pmax = np.array([0.9, 0.9]), np.array([1.1, 1.1])
    pm, ps = np.array([0.0, 1.0]), np.array([0.0, 0.0025])
    cov = np.diag([0.002 ** 2, 0.0025 ** 2])
    s = BatchedMCMC(W, 2, [1, 2], [[1], [2]], 1, pmin, pmax, pm, ps, oversample_fast=oversample,
                    propose_scale=2.4, seed_ij=71, seed_kl=72)
    s.set_covariance(cov)
    s.add_likelihood(like, theory)
    s.set_trial_theory(0, trial)
    s.set_start(np.tile([1.0, 1.0], (W, 1)))
    with pytest.raises(NativeError):
        s.step(1, fast_only=False)              # slow proposals need the trial theory

    def theory_fn(P_trial):
        trial.copy_(base.unsqueeze(0) * P_trial[0].reshape(-1, 1, 1))
    s.step_theory(steps, theory_fn=theory_fn)
    P, lk, mult, nacc = s.state()
    assert np.any(np.abs(P[:, 0] - 1.0) > 1e-6), "no slow move was accepted"
    th, b = theory.cpu().numpy(), base.cpu().numpy()
    orc = po.PlikLite(data)
    bh = np.ascontiguousarray(syn.base_theory(2508)[:3])
    for w in (0, 1, 41, 79):
        np.testing.assert_allclose(th[w], P[w, 0] * b, rtol=1e-15, atol=0)
        ij, kl = walker_seed(71, 72, w)
        h = po.lib().orc_proposer_create(2, np.array([1, 1], dtype=np.int32), np.array([1, 2], dtype=np.int32),
                                         1, oversample, 2.4, 2, np.array([1, 2], dtype=np.int32))
        po.lib().orc_proposer_set_covariance(h, np.ascontiguousarray(cov))
        t = po.Target()
        keep = [np.ascontiguousarray(a) for a in (pmin, pmax, pm, ps)]
        t.num_params = 2
        t.pmin, t.pmax, t.prior_mean, t.prior_std = [a.ctypes.data for a in keep]
        t.temperature = 1.0
        t.plik, t.plik_nuis_index, t.plik_dl, t.plik_ld_field = orc.h, 2, bh.ctypes.data, bh.shape[1]
        t.plik_scale_index = 1
        r = po.Ranmar(ij, kl)
        Q = np.array([1.0, 1.0])
        cur = C.c_double(po.lib().orc_target_loglike(C.byref(t), Q))
        acc = 0
        for _ in range(steps):
            acc += po.lib().orc_mh_step(h, C.byref(r.s), C.byref(t), Q, C.byref(cur), 0, None)
        po.lib().orc_proposer_free(h)
        np.testing.assert_allclose(P[w], Q, rtol=1e-11)
        assert lk[w] == pytest.approx(cur.value, rel=1e-9)


def test_chain_files_from_history(tmp_path):
    """ChainWriter on a GPU run: per walker the weights add up to the steps,
    consecutive rows are distinct points, and the last row is the final state."""
    from cosmomc_amd.chains import ChainWriter
    from cosmomc_amd.sampler import BatchedMCMC
    n, W, T = 2, 8, 90
    s = BatchedMCMC(W, n, [1, 2], [[1, 2]], 1, [-10, -10], [10, 10], seed_ij=5, seed_kl=6)
    s.set_covariance(np.eye(2))
    s.set_test_gaussian(np.array([[1.0, 0.3], [0.3, 2.0]]), np.zeros(2))
    s.set_start(np.zeros((W, n)))
    s.enable_history(40)
    cw = ChainWriter(str(tmp_path / "run"), ["x", "y"], burn_in=-1)
    for _ in range(3):
        s.step(30)
        cw.append(s)
    P, like, mult, _ = s.state()
    open_runs = {w: c for w, c in cw.pending.items()}
    cw.close()
    for w in range(W):
        c = np.loadtxt(tmp_path / f"run_{w + 1}.txt", ndmin=2)
        assert c[:, 0].sum() + open_runs[w][1] == T
        assert open_runs[w][1] == mult[w]                      # the open stay is the sampler's multiplicity
        assert np.all(np.any(np.diff(c[:, 2:], axis=0) != 0, axis=1))
        np.testing.assert_allclose(open_runs[w][0][1:], P[w], rtol=1e-15)
        assert open_runs[w][0][0] == pytest.approx(like[w], rel=1e-15)


def test_interleaved_nuisance_indices(tmp_path):
    """Two likelihoods whose nuisance_indices are not contiguous and not in
    parameter order (GeneralTypes.f90:642-646): plik_lite TTTEEE reads P(4),
    plik_lite TT reads P(2); the fixed parameters between them are never
    passed.  Every walker's CurLike and per-likelihood terms equal the oracle's
    at its final point."""
    from cosmomc_amd.likelihood import NativeCMBLikelihood
    from cosmomc_amd.sampler import BatchedMCMC
    data = syn.make_plik_lite(12345)
    ds = data.write(str(tmp_path))
    l1 = NativeCMBLikelihood("PLIK_LITE", ds)
    l2 = NativeCMBLikelihood("PLIK_LITE", ds, {"use_cl": "TT"})
    l1.nuisance_indices, l2.nuisance_indices = [4], [2]
    W, steps = 130, 30
    th = syn.walker_theory(W, seed=21, n_fields=3)
    dl = torch.tensor(th, device="cuda")
    P0 = np.array([7.0, 1.0, -3.0, 1.0, 5.0])
    pmin = np.array([7.0, 0.9, -3.0, 0.9, 5.0])
    pmax = np.array([7.0, 1.1, -3.0, 1.1, 5.0])
    pm, ps = np.array([0, 1.0, 0, 1.0, 0]), np.array([0, 0.0025, 0, 0.003, 0])
    s = BatchedMCMC(W, 5, [2, 4], [[1], [2]], 0, pmin, pmax, pm, ps, seed_ij=31, seed_kl=32)
    s.set_covariance(np.diag([0.002 ** 2, 0.002 ** 2]))
    s.add_likelihood(l1, dl)
    s.add_likelihood(l2, dl)
    s.enable_history(steps)
    s.set_start(np.tile(P0, (W, 1)))
    s.step(steps, fast_only=True)
    P, lk, _, nacc = s.state()
    assert np.all(nacc > 0)
    terms = s.history_terms(steps - 1, 1)[0]
    o1, o2 = po.PlikLite(data), po.PlikLite(data, use_cl="TT")
    for w in (0, 1, 64, 129):
        t1, t2 = o1.loglike(th[w], P[w, 3]), o2.loglike(th[w], P[w, 1])
        pri = 0.5 * (((P[w, 1] - 1) / 0.0025) ** 2 + ((P[w, 3] - 1) / 0.003) ** 2)
        assert terms[0, w] == pytest.approx(t1, rel=1e-9)
        assert terms[1, w] == pytest.approx(t2, rel=1e-9)
        assert lk[w] == pytest.approx(t1 + t2 + pri, rel=1e-9)


@pytest.mark.parametrize("shared_theory", [True, False])
def test_change_mask_matches_dense(cmbl_golden, refdata, tmp_path, shared_theory):
    """Per-likelihood change mask (LogLikeWithTheorySet, calclike.f90:374-386):
    plik_lite (calPlanck) + BICEP/Keck/Planck (6 varying foreground parameters)
    in separate fast blocks, so every step each walker re-evaluates only the
    likelihood whose parameters moved; the sparse path compacts those walkers
    (plik and the HL CMBlikes kernels on compacted slots, theory rows gathered
    when they are per walker).  Walker groups (cmbs_set_groups) take the dense
    path, which evaluates every likelihood for every walker: both runs must
    make the same accept decisions and end at the same points and terms."""
    import os
    from cosmomc_amd.likelihood import NativeCMBLikelihood
    from cosmomc_amd.sampler import BatchedMCMC
    bc = cmbl_golden["cases"]["bkplanck_3map_bins1to5"]
    plik = NativeCMBLikelihood("PLIK_LITE", syn.make_plik_lite(12345).write(str(tmp_path)))
    bk = NativeCMBLikelihood(bc["tag"], os.path.join(refdata, bc["dataset"]), bc["overrides"])
    plik.nuisance_indices = [2]
    bk.nuisance_indices = list(range(3, 19))
    W, steps = 130, 24
    th = syn.walker_theory(1 if shared_theory else W, seed=8, n_fields=10, ld_field=2512)
    dl = torch.tensor(th, device="cuda")
    if shared_theory:
        dl = dl.expand(W, -1, -1)                     # ld_walker = 0: one slow point
    bk0 = np.array(bc["nuis"][0])
    bk0[1] = 0.5                                      # Async > 0
    P0 = np.concatenate([[0.0222, 1.0], bk0])
    vary = [2, 3, 4, 5, 6, 8, 9]                      # calPlanck, Adust, Async, alphadust, betadust, alphasync, betasync
    pmin, pmax = P0.copy(), P0.copy()
    for i, wdt in zip(vary, [0.1, 2.0, 1.0, 0.5, 0.5, 1.0, 1.0]):
        pmin[i - 1], pmax[i - 1] = P0[i - 1] - wdt, P0[i - 1] + wdt
    pm, ps = np.zeros(18), np.zeros(18)
    pm[1], ps[1] = 1.0, 0.0025
    sig = np.array([0.002, 0.1, 0.05, 0.02, 0.02, 0.05, 0.05])
    runs = []
    for g in (1, 2):
        s = BatchedMCMC(W, 18, vary, [[1], [2, 3, 4, 5, 6, 7]], 0, pmin, pmax, pm, ps, seed_ij=41, seed_kl=42)
        s.set_covariance(np.diag(sig ** 2))
        s.set_groups(g)
        s.add_likelihood(plik, dl)
        s.add_likelihood(bk, dl)
        s.enable_history(steps)
        s.set_start(np.tile(P0, (W, 1)))
        s.step(steps, fast_only=True)
        P, lk, mult, nacc = s.state()
        runs.append((P.copy(), lk.copy(), mult.copy(), nacc.copy(), s.history_terms(0, steps)))
        s.close()
    a, b = runs
    assert np.all(a[3] > 0)
    np.testing.assert_array_equal(a[3], b[3])
    np.testing.assert_array_equal(a[2], b[2])
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])
    np.testing.assert_array_equal(a[4], b[4])
    np.testing.assert_allclose(a[4], b[4], rtol=1e-10)
    # the terms at the final points are the oracles' values there
    import cmblikes_oracle as co
    ob = co.CMBLikesOracle(os.path.join(refdata, bc["dataset"]), bc["overrides"], bc["tag"])
    op = po.PlikLite(syn.make_plik_lite(12345))
    for w in (0, 77, W - 1):
        t = th[0 if shared_theory else w]
        assert a[4][-1, 0, w] == pytest.approx(op.loglike(t, a[0][w, 1]), rel=1e-9)
        assert a[4][-1, 1, w] == pytest.approx(ob.loglike(t, a[0][w, 2:]), rel=1e-9)


@pytest.mark.parametrize("W", [1, 100, 512, 1024])
def test_fused_window_pass(cmbl_golden, refdata, tmp_path, W):
    """plik_lite and the Planck lensing likelihood on one theory buffer run
    their window stages as one pass over it (theorypass.hip; the lensing
    windows are re-segmented where no plik bin is split).  The per-likelihood
    terms of the recorded points equal each likelihood's own loglike_batch
    (rtol 1e-12: only the summation split differs) and the oracles'.
    W = 1024 runs the bench's block plan (16 walker tiles placed by cost),
    W = 1 a single tile; every W runs the slot-reusing columns."""
    import os

    import cmblikes_oracle as co
    from cosmomc_amd import _native as N
    from cosmomc_amd.likelihood import NativeCMBLikelihood
    from cosmomc_amd.sampler import BatchedMCMC
    c = cmbl_golden["cases"]["lensing_consext8"]
    data = syn.make_plik_lite(12345)
    plik = NativeCMBLikelihood("PLIK_LITE", data.write(str(tmp_path)))
    lens = NativeCMBLikelihood(c["tag"], os.path.join(refdata, c["dataset"]), c["overrides"])
    plik.nuisance_indices = [2]
    lens.nuisance_indices = [2]
    steps = 10
    th = syn.walker_theory(W, seed=7, n_fields=10, ld_field=2512)
    dl = torch.tensor(th, device="cuda")
    s = BatchedMCMC(W, 3, [2], [[1]], 0, [0.0222, 0.9, 3.05], [0.0222, 1.1, 3.05], [0.0, 1.0, 0.0],
                    [0.0, 0.0025, 0.0], seed_ij=58, seed_kl=69)
    s.set_covariance(np.array([[0.002 ** 2]]))
    s.add_likelihood(plik, dl)
    s.add_likelihood(lens, dl)
    assert N.lib().cmamd_debug_fused(s._h) > 0, N.lib().cmamd_debug_fused(s._h)
    s.enable_history(steps)
    s.set_start(np.tile([0.0222, 1.0, 3.05], (W, 1)))
    s.step(steps, fast_only=True)
    hist = s.history_host(0, steps)
    terms = s.history_terms(0, steps)
    po_plik = po.PlikLite(data)
    o_lens = co.CMBLikesOracle(os.path.join(refdata, c["dataset"]), c["overrides"], c["tag"])
    for k in (0, steps - 1):
        cal = hist[k, 0, :].copy()
        nu = torch.tensor(cal, device="cuda").reshape(-1, 1)
        np.testing.assert_allclose(terms[k, 0], plik.loglike_batch(dl, nu).cpu().numpy(), rtol=1e-12)
        np.testing.assert_allclose(terms[k, 1], lens.loglike_batch(dl, nu).cpu().numpy(), rtol=1e-12)
        for w in (0, W // 2, W - 1):
            assert terms[k, 0, w] == pytest.approx(po_plik.loglike(th[w, :3], cal[w]), rel=1e-9)
            assert terms[k, 1, w] == pytest.approx(o_lens.loglike(th[w], cal[w:w + 1]), rel=1e-10)


@pytest.mark.parametrize("W", [1, 100, 1024])
def test_corun_tails_bitwise(cmbl_golden, refdata, tmp_path, W):
    """After the fused pass, the lensing chi^2 runs inside plik's deferred
    quadratic-form launch (quadform_corun): the chains, CurLike and both
    likelihood terms are bit-identical to the two separate launches
    (cmamd_debug_corun off), and the terms equal each likelihood's own
    loglike_batch at the recorded points."""
    import os

    from cosmomc_amd import _native as N
    from cosmomc_amd.likelihood import NativeCMBLikelihood
    from cosmomc_amd.sampler import BatchedMCMC
    c = cmbl_golden["cases"]["lensing_consext8"]
    data = syn.make_plik_lite(12345)
    th = syn.walker_theory(W, seed=9, n_fields=10, ld_field=2512)
    dl = torch.tensor(th, device="cuda")
    steps = 8
    out = []
    for corun in (1, 0):
        plik = NativeCMBLikelihood("PLIK_LITE", data.write(str(tmp_path)))
        lens = NativeCMBLikelihood(c["tag"], os.path.join(refdata, c["dataset"]), c["overrides"])
        plik.nuisance_indices = [2]
        lens.nuisance_indices = [2]
        s = BatchedMCMC(W, 3, [2], [[1]], 0, [0.0222, 0.9, 3.05], [0.0222, 1.1, 3.05], [0.0, 1.0, 0.0],
                        [0.0, 0.0025, 0.0], seed_ij=59, seed_kl=70)
        s.set_covariance(np.array([[0.002 ** 2]]))
        s.add_likelihood(plik, dl)
        s.add_likelihood(lens, dl)
        assert N.lib().cmamd_debug_fused(s._h) > 0
        assert N.lib().cmamd_debug_corun(s._h, corun) == 0
        s.enable_history(steps)
        s.set_start(np.tile([0.0222, 1.0, 3.05], (W, 1)))
        s.step(steps, fast_only=True)
        out.append((s.history_host(0, steps), s.history_terms(0, steps)))
        if corun:
            cal = out[0][0][steps - 1, 0, :].copy()
            nu = torch.tensor(cal, device="cuda").reshape(-1, 1)
            np.testing.assert_allclose(out[0][1][steps - 1, 1], lens.loglike_batch(dl, nu).cpu().numpy(),
                                       rtol=1e-12)
    assert np.array_equal(out[0][0], out[1][0])
    assert np.array_equal(out[0][1], out[1][1])


@pytest.mark.parametrize("W", [1, 100, 1024])
def test_pipelined_steps_bitwise(cmbl_golden, refdata, tmp_path, W):
    """The fast-step schedules give the same bits.  Mode 3 (the default, the
    unified step launch): one launch per step holds step k's quadratic form
    and lensing chi^2, the pass storing step k + 1's raw sums, and the
    Metropolis workgroups that wait for their tile's tails, accept step k and
    propose step k + 1 (mh_step_kernel).  Mode 0: the unpipelined schedule.
    Each runs the lean Metropolis chain (mhlean.h: the only fast parameter is
    a one-parameter block) and the generic chain (mh_body), which the
    reference chains pin.  Chains, CurLike and both likelihood terms are
    bit-identical over step() calls of 1, 2 and 5 steps.  The default
    schedule's own run is pinned to the oracles directly: at the first and
    last recorded steps the terms of walkers 0, W/2 - 1 and W - 1 equal
    pyoracle.PlikLite's and CMBLikesOracle's -lnL at the recorded calibrations
    (rel 1e-9), and every walker's equals each likelihood's own loglike_batch
    (rtol 1e-12)."""
    import os

    import cmblikes_oracle as co
    from cosmomc_amd import _native as N
    from cosmomc_amd.likelihood import NativeCMBLikelihood
    from cosmomc_amd.sampler import BatchedMCMC
    c = cmbl_golden["cases"]["lensing_consext8"]
    data = syn.make_plik_lite(12345)
    th = syn.walker_theory(W, seed=11, n_fields=10, ld_field=2512)
    dl = torch.tensor(th, device="cuda")
    calls = (1, 2, 5)
    steps = sum(calls)
    out = []
    for mode, lean in ((-1, 1), (3, 1), (0, 1), (3, 0), (0, 0)):
        plik = NativeCMBLikelihood("PLIK_LITE", data.write(str(tmp_path)))
        lens = NativeCMBLikelihood(c["tag"], os.path.join(refdata, c["dataset"]), c["overrides"])
        plik.nuisance_indices = [2]
        lens.nuisance_indices = [2]
        s = BatchedMCMC(W, 3, [2], [[1]], 0, [0.0222, 0.9, 3.05], [0.0222, 1.1, 3.05], [0.0, 1.0, 0.0],
                        [0.0, 0.0025, 0.0], seed_ij=61, seed_kl=72)
        s.set_covariance(np.array([[0.002 ** 2]]))
        s.add_likelihood(plik, dl)
        s.add_likelihood(lens, dl)
        assert N.lib().cmamd_debug_fused(s._h) > 0
        if mode >= 0:                                     # -1: the default schedule
            assert N.lib().cmamd_debug_pipeline(s._h, mode) == 0
        assert N.lib().cmamd_debug_lean(s._h, lean) == 0
        s.enable_history(steps)
        s.set_start(np.tile([0.0222, 1.0, 3.05], (W, 1)))
        for n in calls:
            s.step(n, fast_only=True)
        if mode != 0:
            assert N.lib().cmamd_debug_tail(s._h) == W        # the unified launch ran
        out.append((s.history_host(0, steps), s.history_terms(0, steps)))
        assert plik.status() == 0 and lens.status() == 0
        if mode == -1:
            po_plik = po.PlikLite(data)
            o_lens = co.CMBLikesOracle(os.path.join(refdata, c["dataset"]), c["overrides"], c["tag"])
            for k in (0, steps - 1):
                cal = out[0][0][k, 0, :].copy()
                nu = torch.tensor(cal, device="cuda").reshape(-1, 1)
                np.testing.assert_allclose(out[0][1][k, 0], plik.loglike_batch(dl, nu).cpu().numpy(), rtol=1e-12)
                np.testing.assert_allclose(out[0][1][k, 1], lens.loglike_batch(dl, nu).cpu().numpy(), rtol=1e-12)
                for w in sorted({0, max(0, W // 2 - 1), W - 1}):
                    assert out[0][1][k, 0, w] == pytest.approx(po_plik.loglike(th[w, :3], cal[w]), rel=1e-9)
                    assert out[0][1][k, 1, w] == pytest.approx(o_lens.loglike(th[w], cal[w:w + 1]), rel=1e-9)
        s.close()
    for o in out[1:]:
        assert np.array_equal(out[0][0], o[0])
        assert np.array_equal(out[0][1], o[1])


def test_pipelined_with_wide_slow_block(cmbl_golden, refdata, tmp_path):
    """A slow block wide enough for rot_kernel's rotations (9 parameters) does
    not keep fast-only steps off the pipelined schedule (fast-only steps never
    propose it): the unified step launch runs (mode 3) and the chains equal
    the unpipelined steps' (mode 0) bit for bit."""
    import os

    from cosmomc_amd import _native as N
    from cosmomc_amd.likelihood import NativeCMBLikelihood
    from cosmomc_amd.sampler import BatchedMCMC
    c = cmbl_golden["cases"]["lensing_consext8"]
    W, n = 256, 10
    data = syn.make_plik_lite(12345)
    th = syn.walker_theory(W, seed=13, n_fields=10, ld_field=2512)
    dl = torch.tensor(th, device="cuda")
    P0 = np.concatenate([np.linspace(0.1, 0.9, n - 1), [1.0]])
    pmin, pmax = P0 - 1.0, P0 + 1.0
    pmin[-1], pmax[-1] = 0.9, 1.1
    pm, ps = np.zeros(n), np.zeros(n)
    pm[-1], ps[-1] = 1.0, 0.0025
    out = []
    for mode in (3, 0):
        plik = NativeCMBLikelihood("PLIK_LITE", data.write(str(tmp_path)))
        lens = NativeCMBLikelihood(c["tag"], os.path.join(refdata, c["dataset"]), c["overrides"])
        plik.nuisance_indices = [n]
        lens.nuisance_indices = [n]
        s = BatchedMCMC(W, n, list(range(1, n + 1)), [list(range(1, n)), [n]], 1, pmin, pmax, pm, ps,
                        seed_ij=81, seed_kl=92)
        s.set_covariance(np.diag(np.concatenate([np.full(n - 1, 0.01), [0.002]]) ** 2))
        s.add_likelihood(plik, dl)
        s.add_likelihood(lens, dl)
        assert N.lib().cmamd_debug_pipeline(s._h, mode) == 0
        s.enable_history(12)
        s.set_start(np.tile(P0, (W, 1)))
        N.profile_enable(True)
        N.profile_reset()
        s.step(5, fast_only=True)
        s.step(7, fast_only=True)
        torch.cuda.synchronize()
        launches = N.profile_read("mh_step_kernel")[1]
        N.profile_enable(False)
        assert (launches == 10) if mode == 3 else (launches == 0)   # the middle launches of the two calls
        out.append((s.history_host(0, 12), s.history_terms(0, 12), s.save_state()))
        s.close()
    assert np.array_equal(out[0][0], out[1][0])
    assert np.array_equal(out[0][1], out[1][1])
    assert out[0][2] == out[1][2]


@pytest.mark.parametrize("mode", [3, "bin"])
def test_pipelined_handoff_giveup_fails_loudly(cmbl_golden, refdata, tmp_path, mode):
    """In-launch hand-offs fail loudly.  Mode 3: the unified step launch's
    Metropolis workgroups wait for their tile's tails; "bin": mh_bin_kernel's
    bin workgroups wait for the calibrations the Metropolis workgroups
    publish.  A debug switch stops the producers (no arrivals / no
    publication), so every wait gives up at its bound and sets
    CMBL_STATUS_PIPE_WAIT; the next readback (and the next step call) must fail
    instead of handing back silently rejected trials."""
    import os

    from cosmomc_amd import _native as N
    from cosmomc_amd.likelihood import NativeCMBLikelihood
    from cosmomc_amd.sampler import BatchedMCMC
    c = cmbl_golden["cases"]["lensing_consext8"]
    W = 128
    th = syn.walker_theory(W, seed=12, n_fields=10, ld_field=2512)
    dl = torch.tensor(th, device="cuda")
    plik = NativeCMBLikelihood("PLIK_LITE", syn.make_plik_lite(12345).write(str(tmp_path)))
    lens = NativeCMBLikelihood(c["tag"], os.path.join(refdata, c["dataset"]), c["overrides"])
    plik.nuisance_indices = [2]
    lens.nuisance_indices = [2]
    s = BatchedMCMC(W, 3, [2], [[1]], 0, [0.0222, 0.9, 3.05], [0.0222, 1.1, 3.05], [0.0, 1.0, 0.0],
                    [0.0, 0.0025, 0.0], seed_ij=63, seed_kl=74)
    s.set_covariance(np.array([[0.002 ** 2]]))
    s.add_likelihood(plik, dl)
    if mode != "bin":   # "bin": plik alone, the bin co-run's bins wait for the calibrations
        s.add_likelihood(lens, dl)
    assert N.lib().cmamd_debug_pipeline(s._h, 3) == 0
    s.set_start(np.tile([0.0222, 1.0, 3.05], (W, 1)))
    s.step(2, fast_only=True)                                  # healthy
    s.state()
    assert N.lib().cmamd_debug_tail_nosignal(s._h, 1) == 0
    s.step(2, fast_only=True)                                  # every wait gives up
    with pytest.raises(Exception, match="gave up"):
        s.state()
    assert N.lib().cmamd_debug_tail_nosignal(s._h, 0) == 0
    s.close()


def test_dragging_fused_plik_lensing(cmbl_golden, refdata, tmp_path):
    """Dragging with plik_lite + lensing on one theory buffer (the fused
    window pass at both the start and the end-point theories): every walker's
    final theory row is A_w x base and its terms are the oracles' there."""
    import os

    import cmblikes_oracle as co
    from cosmomc_amd import _native as N
    from cosmomc_amd.likelihood import NativeCMBLikelihood
    from cosmomc_amd.sampler import BatchedMCMC
    c = cmbl_golden["cases"]["lensing_consext8"]
    data = syn.make_plik_lite(12345)
    plik = NativeCMBLikelihood("PLIK_LITE", data.write(str(tmp_path)))
    lens = NativeCMBLikelihood(c["tag"], os.path.join(refdata, c["dataset"]), c["overrides"])
    plik.nuisance_indices = [2]
    lens.nuisance_indices = [2]
    W = 130
    base = torch.tensor(syn.walker_theory(1, seed=4, n_fields=10, ld_field=2512), device="cuda")[0]
    theory = base.unsqueeze(0).repeat(W, 1, 1).contiguous()
    end = torch.empty_like(theory)
    pmin, pmax = np.array([0.95, 0.9]), np.array([1.05, 1.1])
    pm, ps = np.array([0.0, 1.0]), np.array([0.0, 0.0025])
    s = BatchedMCMC(W, 2, [1, 2], [[1], [2]], 1, pmin, pmax, pm, ps, propose_scale=2.4, seed_ij=93, seed_kl=94)
    s.set_covariance(np.diag([0.002 ** 2, 0.0025 ** 2]))
    s.add_likelihood(plik, theory)
    s.add_likelihood(lens, theory)
    assert N.lib().cmamd_debug_fused(s._h) > 0
    s.set_drag_theory(0, end)
    s.set_drag_theory(1, end)
    s.set_start(np.tile([1.0, 1.0], (W, 1)))
    s.enable_history(64)

    def theory_fn(P_end):
        torch.mul(base.unsqueeze(0), P_end[0].reshape(-1, 1, 1), out=end)
    s.step_drag(12, theory_fn=theory_fn)
    P, lk, mult, nacc = s.state()
    terms = s.history_terms(s.history_count() - 1, 1)[0]
    assert np.any(np.abs(P[:, 0] - 1.0) > 1e-6), "no drag was accepted"
    th = theory.cpu().numpy()
    b = base.cpu().numpy()
    op = po.PlikLite(data)
    ol = co.CMBLikesOracle(os.path.join(refdata, c["dataset"]), c["overrides"], c["tag"])
    for w in (0, 64, W - 1):
        np.testing.assert_allclose(th[w], P[w, 0] * b, rtol=1e-15, atol=0)
        assert terms[0, w] == pytest.approx(op.loglike(th[w, :3], P[w, 1]), rel=1e-9)
        assert terms[1, w] == pytest.approx(ol.loglike(th[w], P[w, 1:2]), rel=1e-10)
        ref = terms[0, w] + terms[1, w] + 0.5 * ((P[w, 1] - 1.0) / 0.0025) ** 2
        assert lk[w] == pytest.approx(ref, rel=1e-12)


@pytest.mark.parametrize("W", [130, 1024])
def test_drag_staged_matches_hbm(cmbl_golden, refdata, tmp_path, W):
    """The drag stages on an LDS image of the walkers' state (drag_staged_kernel,
    the default) and on the HBM state (drag_kernel), and the interpolation
    steps' two evaluation sets paired into two launches (theory_window_pair +
    quadform_pair_ticket, the default) or run one after the other, give the
    same chains bit for bit: history rows, terms and the final state."""
    import os

    from cosmomc_amd import _native as N
    from cosmomc_amd.likelihood import NativeCMBLikelihood
    from cosmomc_amd.sampler import BatchedMCMC
    c = cmbl_golden["cases"]["lensing_consext8"]
    data = syn.make_plik_lite(12345)
    base = torch.tensor(syn.walker_theory(1, seed=4, n_fields=10, ld_field=2512), device="cuda")[0]
    out = []
    for hbm, pair in ((0, 1), (1, 1), (0, 0)):
        plik = NativeCMBLikelihood("PLIK_LITE", data.write(str(tmp_path)))
        lens = NativeCMBLikelihood(c["tag"], os.path.join(refdata, c["dataset"]), c["overrides"])
        plik.nuisance_indices = [2]
        lens.nuisance_indices = [2]
        theory = base.unsqueeze(0).repeat(W, 1, 1).contiguous()
        end = torch.empty_like(theory)
        s = BatchedMCMC(W, 2, [1, 2], [[1], [2]], 1, np.array([0.95, 0.9]), np.array([1.05, 1.1]),
                        np.array([0.0, 1.0]), np.array([0.0, 0.0025]), propose_scale=2.4, seed_ij=95, seed_kl=96)
        s.set_covariance(np.diag([0.002 ** 2, 0.0025 ** 2]))
        s.add_likelihood(plik, theory)
        s.add_likelihood(lens, theory)
        assert N.lib().cmamd_debug_drag_hbm(s._h, hbm) == 0
        assert N.lib().cmamd_debug_drag_pair(s._h, pair) == 0
        s.set_drag_theory(0, end)
        s.set_drag_theory(1, end)
        s.set_start(np.tile([1.0, 1.0], (W, 1)))
        s.enable_history(64)

        def theory_fn(P_end):
            torch.mul(base.unsqueeze(0), P_end[0].reshape(-1, 1, 1), out=end)
        s.step_drag(10, theory_fn=theory_fn)
        n = s.history_count()
        out.append((s.history_host(0, n), s.history_terms(0, n), *s.state()))
        s.close()
    a = out[0]
    assert np.any(a[5] > 0), "no drag was accepted"
    for b in out[1:]:
        for x, y in zip(a, b):
            assert np.array_equal(x, y)


@pytest.mark.parametrize("blocks,W,groups", [([21], 512, 1), ([12, 9], 576, 1), ([32], 200, 1), ([8, 13], 320, 2)])
def test_parallel_rotations_match_serial(blocks, W, groups):
    """rot_kernel's parallel rotation (64-lane RANMAR rounds, ballot-placed
    Gaussian1 pairs, lockstep Gram-Schmidt, exact state commit) leaves every
    walker's whole state -- R, the RANMAR ring and pointers, c, iset/gset,
    points and likelihoods -- bit-identical to the serial path (lane 0 draws
    one Gaussian at a time), over several rotations per walker, including the
    redraws of rows whose norm falls below 1e-3 (about 2.5 % of the 21-d
    rotations: taken by the spare lanes' attempts, or, in debug mode 2, by
    restarting the pass) and blocks of 8 (ROT_DEFER_MIN) to 32 (MAXBLK)
    parameters."""
    from cosmomc_amd import _native as N
    from cosmomc_amd.sampler import BatchedMCMC
    n = sum(blocks)
    rng = np.random.default_rng(n + W)
    width = rng.uniform(0.05, 2.0, n)
    A = rng.standard_normal((n, n))
    cov = (A @ A.T / n + np.eye(n)) * np.outer(width, width) / 2
    P0 = rng.uniform(-1.0, 1.0, n)
    used = list(range(1, n + 1))
    split, k = [], 0
    for b in blocks:
        split.append(used[k:k + b])
        k += b
    steps = 3 * max(blocks) + 2
    start = np.tile(P0, (W, 1)) + 0.1 * rng.standard_normal((W, n)) * width
    images = []
    for serial in (0, 1, 2):
        s = BatchedMCMC(W, n, used, split, 0, P0 - 20 * width, P0 + 20 * width, propose_scale=2.4,
                        seed_ij=4004, seed_kl=9373)
        s.set_covariance(np.diag(width ** 2))
        s.set_test_gaussian(cov, P0)
        if groups > 1:
            s.set_groups(groups)
        assert N.lib().cmamd_debug_rot_serial(s._h, serial) == 0
        s.set_start(start)
        for _ in range(steps):
            s.step(1, fast_only=True)
        images.append((s.save_state(), s.state()))
        s.close()
    (a, sa), (b, sb), (c, sc) = images
    np.testing.assert_array_equal(sa[0], sb[0])
    np.testing.assert_array_equal(sa[1], sb[1])
    assert a == b
    assert c == b          # mode 2: a last-row redraw restarts the pass instead of using the spare lanes


@pytest.mark.parametrize("blocks,W,force", [([21], 512, 1), ([12, 9], 320, 1), ([4, 17], 256, 0)])
def test_rotation_rows_in_place_match_staged(blocks, W, force):
    """The rotation rows in HBM (set_mh_lds's choice when rot_kernel draws
    every rotation wider than one parameter; the only fast block's next column
    fetched by the thread groups beside the image) and staged in mh_kernel's
    LDS image leave every walker's whole state bit-identical, over several
    rotations per walker, rotating steps (rot_kernel) and fast-only steps
    alike; [4, 17] forces the in-place rows with a 4-wide block rotating inside
    the chain (below ROT_DEFER_MIN)."""
    from cosmomc_amd import _native as N
    from cosmomc_amd.sampler import BatchedMCMC
    n = sum(blocks)
    rng = np.random.default_rng(7 * n + W)
    width = rng.uniform(0.05, 2.0, n)
    A = rng.standard_normal((n, n))
    cov = (A @ A.T / n + np.eye(n)) * np.outer(width, width) / 2
    P0 = rng.uniform(-1.0, 1.0, n)
    used = list(range(1, n + 1))
    split, k = [], 0
    for b in blocks:
        split.append(used[k:k + b])
        k += b
    start = np.tile(P0, (W, 1)) + 0.1 * rng.standard_normal((W, n)) * width
    images = []
    for mode in (-1, force):
        s = BatchedMCMC(W, n, used, split, 0, P0 - 20 * width, P0 + 20 * width, propose_scale=2.4,
                        seed_ij=4114, seed_kl=9373)
        s.set_covariance(np.diag(width ** 2))
        s.set_test_gaussian(cov, P0)
        assert N.lib().cmamd_debug_stage_R(s._h, mode) == 0
        s.set_start(start)
        s.step(2 * max(blocks) + 3, fast_only=True)
        s.step(3, fast_only=False)
        s.step(max(blocks), fast_only=True)
        images.append((s.save_state(), s.state()))
        s.close()
    (a, sa), (b, sb) = images
    assert np.any(sa[3] > 0)
    for x, y in zip(sa, sb):
        np.testing.assert_array_equal(x, y)
    assert a == b


@pytest.mark.parametrize("W,shared", [(512, True), (200, False)])
def test_bin_corun_bitwise(tmp_path, W, shared):
    """The bin co-run (config4_fast21's schedule: plik_lite binned into raw
    sums inside the proposing launch, its quadratic form forming Delta = X -
    S / cal^2 from them) leaves every walker's state, history row and
    likelihood terms bit-identical to the unpipelined steps (plik_bin_delta +
    quadform_ksplit), across the 21-wide block's rotations (rot_kernel between
    the proposing launch and the quadratic form); the walkers' terms match
    the plik_lite oracle."""
    from cosmomc_amd import _native as N
    from cosmomc_amd.likelihood import NativeCMBLikelihood
    from cosmomc_amd.sampler import BatchedMCMC
    n = 21
    data = syn.make_plik_lite(12345)
    rng = np.random.default_rng(2121)
    width = np.concatenate([[0.0025], rng.uniform(0.05, 2.0, n - 1)])
    A = rng.standard_normal((n - 1, n - 1))
    corr = A @ A.T / (n - 1) + np.eye(n - 1)
    d = np.sqrt(np.diag(corr))
    cov = np.zeros((n, n))
    cov[0, 0] = 1.0
    cov[1:, 1:] = corr / d[:, None] / d[None, :] * np.outer(width[1:], width[1:])
    P0 = np.concatenate([[1.0], rng.uniform(-1.0, 1.0, n - 1)])
    pmin, pmax = P0 - 20 * width, P0 + 20 * width
    pmin[0], pmax[0] = 0.9, 1.1
    pm, ps = np.zeros(n), np.zeros(n)
    pm[0], ps[0] = 1.0, 0.0025
    used = list(range(1, n + 1))
    th = syn.walker_theory(1 if shared else W, seed=5, n_fields=3, ld_field=2512)
    dl = torch.tensor(th, device="cuda")
    if shared:
        dl = dl.expand(W, th.shape[1], th.shape[2])
    g = syn.gaussians(123, W * n).reshape(W, n)
    start = np.clip(P0 + 2 * width * g, pmin + 1e-9, pmax - 1e-9)
    out = []
    for mode in (3, 0):
        plik = NativeCMBLikelihood("PLIK_LITE", data.write(str(tmp_path / f"m{mode}")))
        plik.nuisance_indices = [1]
        smp = BatchedMCMC(W, n, used, [used], 0, pmin, pmax, pm, ps, propose_scale=2.4, seed_ij=4004, seed_kl=9373)
        smp.set_covariance(np.diag(width ** 2))
        smp.set_test_gaussian(cov, P0)
        smp.add_likelihood(plik, dl)
        assert N.lib().cmamd_debug_pipeline(smp._h, mode) == 0
        smp.set_start(start)
        smp.enable_history(64)
        smp.step(25, fast_only=True)
        smp.step(19, fast_only=True)
        k = smp.history_count()
        out.append((smp.history_host(0, k), smp.history_terms(0, k), smp.save_state(), *smp.state()))
        smp.close()
    a, b = out
    assert np.any(a[6] > 0)
    for x, y in zip(a, b):
        if isinstance(x, bytes):
            assert x == y
        else:
            np.testing.assert_array_equal(x, y)
    orc = po.PlikLite(data)
    terms = a[1]
    P = a[3]
    for w in (0, W // 2 - 1, W - 1):   # the last history row's plik term at the walker's point
        ref = orc.loglike(th[0 if shared else w], P[w, 0])
        assert terms[-1, 0, w] == pytest.approx(ref, rel=1e-9)


def _config5_sampler(refdata, tmp_path, W, groups, tdust_free=False):
    """BASELINE configs[4] as bench.py's config5_bk15_plik builds it: BK15 (12
    B maps x 9 bins, HL, batch3/BK15.ini foreground parameters) + plik_lite
    TTTEEE on one shared slow point, 8 fast parameters in the blocks the
    reference's SetFastSlowParams makes (plik_lite, then BK15)."""
    import os

    from cosmomc_amd.likelihood import LikelihoodList, NativeCMBLikelihood
    from cosmomc_amd.params import set_fast_slow_params
    from cosmomc_amd.sampler import BatchedMCMC
    maps = ("BK15_95_B BK15_150_B BK15_220_B W023_B P030_B W033_B P044_B P070_B P100_B P143_B P217_B "
            "P353_B")
    data = syn.make_plik_lite(12345)
    plik = NativeCMBLikelihood("PLIK_LITE", data.write(str(tmp_path)))
    bk = NativeCMBLikelihood("BKPLANCK", os.path.join(refdata, "BK15/BK15_dust.dataset"), {"maps_use": maps})
    plik.nuisance_indices = [1]
    bk.nuisance_indices = list(range(2, 18))
    P0 = np.array([1.0, 3.0, 1.0, -0.42, 1.59, 19.6, -0.6, -3.1, 0.2, 2.0, 2.0, 1.0, 1.0, 0.0, 0.0, 0.0, 0.0])
    pmin, pmax = P0.copy(), P0.copy()
    for i, lo, hi in ((0, 0.9, 1.1), (1, 0.0, 15.0), (2, 0.0, 50.0), (3, -1.0, 0.0), (4, 1.04, 2.14),
                      (6, -1.0, 0.0), (7, -4.5, -2.0), (8, -1.0, 1.0)):
        pmin[i], pmax[i] = lo, hi
    pm, ps = np.zeros(17), np.zeros(17)
    pm[0], ps[0] = 1.0, 0.0025
    pm[4], ps[4] = 1.59, 0.11
    pm[7], ps[7] = -3.1, 0.3
    used = [1, 2, 3, 4, 5, 7, 8, 9]
    width = [0.0025, 0.5, 1.0, 0.1, 0.1, 0.1, 0.3, 0.2]
    if tdust_free:          # T_dust (DataParams(5) of BK15) a fast parameter, different in every walker
        pmin[5], pmax[5] = 15.0, 25.0
        used = [1, 2, 3, 4, 5, 6, 7, 8, 9]
        width.insert(5, 0.5)
    width = np.array(width)
    ll = LikelihoodList()
    ll.add(plik)
    ll.add(bk)
    ll.add_nuisance_parameters([])
    blk = set_fast_slow_params(17, [i + 1 in used for i in range(17)], list(ll), num_theory_params=0)
    s = BatchedMCMC(W, 17, used, blk.param_blocks, blk.slow_block_max, pmin, pmax, pm, ps, propose_scale=2.4,
                    seed_ij=3003, seed_kl=9373)
    s.set_covariance(np.diag(width ** 2))
    s.set_groups(groups)
    th = syn.walker_theory(1, n_fields=10, ld_field=2512)
    dl = torch.tensor(th, device="cuda").expand(W, th.shape[1], th.shape[2])
    s.add_likelihood(plik, dl)
    s.add_likelihood(bk, dl)
    start = np.tile(P0, (W, 1))
    g = syn.gaussians(91, W * len(used)).reshape(W, len(used))
    for c, i in enumerate([u - 1 for u in used]):
        start[:, i] = np.clip(P0[i] + 2 * width[c] * g[:, c], pmin[i] + 1e-9, pmax[i] - 1e-9)
    s.set_start(start)
    return s, data, th[0], maps


def test_config5_joint_path_vs_oracles(refdata, tmp_path):
    """The configs[4] leg exactly as bench.py runs it (BK15 12 B maps + plik_lite,
    W = 1024, 5 fast steps): with the change mask on (one walker group: each
    likelihood re-evaluated only for the walkers whose trial moved one of its
    parameters, the HL kernels on compacted slots) the accept decisions,
    multiplicities, points and -lnL equal the dense path's (two walker groups:
    every likelihood for every walker) bit for bit -- the HL eigensolves stop
    per problem, so a walker's terms do not depend on which walkers share its
    wave -- and the terms at the final points of walkers 0, 511 and 1023 are
    the oracles' (pyoracle.PlikLite, CMBLikesOracle; rel 1e-9)."""
    import os

    import cmblikes_oracle as co
    W, steps = 1024, 5
    runs = []
    for groups in (1, 2):
        s, data, th, maps = _config5_sampler(refdata, tmp_path, W, groups)
        s.enable_history(steps)
        s.step(steps, fast_only=True)
        P, lk, mult, nacc = s.state()
        runs.append((P.copy(), lk.copy(), mult.copy(), nacc.copy(), s.history_terms(0, steps)))
        s.close()
    a, b = runs
    assert a[3].sum() > W // 4                       # walkers did move (about a third of the trials accepted)
    np.testing.assert_array_equal(a[3], b[3])
    np.testing.assert_array_equal(a[2], b[2])
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])
    np.testing.assert_array_equal(a[4], b[4])
    ob = co.CMBLikesOracle(os.path.join(refdata, "BK15/BK15_dust.dataset"), {"maps_use": maps}, "BKPLANCK")
    op = po.PlikLite(data)
    for w in (0, 511, 1023):
        assert a[4][-1, 0, w] == pytest.approx(op.loglike(th[:3], a[0][w, 0]), rel=1e-9)
        assert a[4][-1, 1, w] == pytest.approx(ob.loglike(th, a[0][w, 1:17]), rel=1e-9)


def test_bk_tdust_per_walker_groups_bitwise(refdata, tmp_path):
    """BK15's dust greybody denominators are tabulated per call for the first
    walker's T_dust (cmbl_bk_tdtab) in the call's own workspace.  With T_dust a
    fast parameter that differs between walkers, two and four walker groups
    (each group's BK evaluation on its own stream, concurrently) give the same
    bits as one group, and the final terms are the oracle's (the
    table used to live in the likelihood object, shared across streams)."""
    import os

    import cmblikes_oracle as co
    W, steps = 256, 4
    runs = []
    for groups in (1, 2, 4):
        s, data, th, maps = _config5_sampler(refdata, tmp_path, W, groups, tdust_free=True)
        s.enable_history(steps)
        s.step(steps, fast_only=True)
        P, lk, mult, nacc = s.state()
        runs.append((P.copy(), lk.copy(), mult.copy(), nacc.copy(), s.history_terms(0, steps)))
        s.close()
    a = runs[0]
    assert np.unique(a[0][:, 5]).size > W // 2        # T_dust differs between walkers
    assert a[3].sum() > 0
    for b in runs[1:]:
        for x, y in zip(a, b):
            np.testing.assert_array_equal(x, y)
    ob = co.CMBLikesOracle(os.path.join(refdata, "BK15/BK15_dust.dataset"), {"maps_use": maps}, "BKPLANCK")
    for w in (0, 127, 128, 255):
        assert a[4][-1, 1, w] == pytest.approx(ob.loglike(th, a[0][w, 1:17]), rel=1e-9)


def test_headline_chain_follows_oracle_step_by_step(tmp_path):
    """BASELINE configs[2]'s headline fast step exactly as bench.py builds it
    (plik_lite TTTEEE + Planck 2018 lensing on per-walker theory, calPlanck
    fast with its prior, W = 1024) on the default schedule -- the unified
    launch (mh_step_kernel) with the lean chain -- for 24 steps.  Walkers
    {0, W/2 - 1, W - 1} follow an oracle chain step by step: the C oracle's
    FastParameterSample (orc_mh_step: BlockedProposer, RANMAR, GetLogLike,
    MetropolisAccept) on a target of pyoracle.PlikLite + the CMBlikes numpy
    restatement of the lensing likelihood (LogLikeWithTheorySet,
    calclike.f90:357-389, in list order) + the calPlanck prior.  Every accept
    decision matches, and the point and CurLike after every step match at
    rtol 1e-11 / 1e-9 (MCMC.f90:309-335, calclike.f90:136-151)."""
    import os

    import bench
    import cmblikes_oracle as co
    from cosmomc_amd import _native as N
    from cosmomc_amd.sampler import walker_seed
    W, steps = 1024, 24
    smp, likes, theory, _ = bench.build_problem(W, 0, str(tmp_path))
    smp.enable_history(steps)
    N.profile_enable(True)
    N.profile_reset()
    smp.step(steps, fast_only=True)
    torch.cuda.synchronize()
    assert N.profile_read("mh_step_kernel")[1] == steps - 1     # the unified launch ran every middle step
    N.profile_enable(False)
    rows = smp.history_host(0, steps)                              # [steps, 8, W]: P(1..7), CurLike
    th = theory.cpu().numpy()
    data = syn.make_plik_lite(12345)
    plik = po.PlikLite(data)
    lens = co.CMBLikesOracle(os.path.join(str(tmp_path), "refdata", bench.LENS_DATASET))
    P0 = np.array([0.02237, 0.1200, 1.04092, 0.0544, 3.044, 0.9649, 1.0])
    sig = np.array([0.00015, 0.0012, 0.00031, 0.0073, 0.014, 0.0042, 0.0025])
    pmin, pmax = P0 - 50 * sig, P0 + 50 * sig
    pmin[6], pmax[6] = 0.9, 1.1
    pm, ps = np.zeros(7), np.zeros(7)
    pm[6], ps[6] = 1.0, 0.0025
    keep = [np.ascontiguousarray(a) for a in (pmin, pmax, pm, ps)]
    n_acc_total = 0
    for w in (0, W // 2 - 1, W - 1):
        dlw = np.ascontiguousarray(th[w])
        calls = []

        def lensing_term(user, Pp, dlw=dlw, calls=calls):
            calls.append(1)
            return float(lens.loglike(dlw, np.array([Pp[6]])))
        cb = po.EXTRA_LIKE_FN(lensing_term)
        t = po.Target()
        t.num_params = 7
        t.pmin, t.pmax, t.prior_mean, t.prior_std = [a.ctypes.data for a in keep]
        t.temperature = 1.0
        t.plik, t.plik_nuis_index, t.plik_dl, t.plik_ld_field = plik.h, 7, dlw.ctypes.data, dlw.shape[1]
        t.extra_like = C.cast(cb, C.c_void_p)
        blocks = np.array([1, 2, 3, 4, 5, 6, 7], dtype=np.int32)
        h = po.lib().orc_proposer_create(2, np.array([6, 1], dtype=np.int32), blocks, 1, 1, 2.4, 7,
                                         np.arange(1, 8, dtype=np.int32))
        po.lib().orc_proposer_set_covariance(h, np.ascontiguousarray(np.diag(sig ** 2)))
        r = po.Ranmar(*walker_seed(1802, 9373, w))
        Q = P0.copy()
        cur = C.c_double(po.lib().orc_target_loglike(C.byref(t), Q))
        for k in range(steps):
            prev = rows[k - 1, :7, w] if k else P0
            acc = po.lib().orc_mh_step(h, C.byref(r.s), C.byref(t), Q, C.byref(cur), 1, None)
            moved = not np.array_equal(rows[k, :7, w], prev)
            assert bool(acc) == moved, (w, k)
            n_acc_total += acc
            np.testing.assert_allclose(rows[k, :7, w], Q, rtol=1e-11, atol=0, err_msg=f"walker {w} step {k}")
            assert rows[k, 7, w] == pytest.approx(cur.value, rel=1e-9), (w, k)
        po.lib().orc_proposer_free(h)
        assert steps // 2 < len(calls) <= steps + 1     # trials out of bounds never reach the likelihoods
    assert n_acc_total > 10
    smp.close()


def test_binned_cache_same_bits(tmp_path):
    """cmbs_set_binned_cache: the unified fast step binning each walker's
    theory once per call and reusing the raw sums gives the same chains,
    history rows and terms bit for bit as re-binning at every step (the
    theory is fixed inside a call; the sums are calibration-independent)."""
    import bench
    W = 256
    out = []
    for cache in (False, True):
        smp, likes, theory, _ = bench.build_problem(W, 0, str(tmp_path / f"c{int(cache)}"))
        smp.set_binned_cache(cache)
        smp.enable_history(40)
        smp.step(15, fast_only=True)
        smp.step(9, fast_only=True)
        k = smp.history_count()
        out.append((smp.history_host(0, k), smp.history_terms(0, k), *smp.state()))
        smp.close()
    a, b = out
    assert np.any(a[5] > 0)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
