"""Checkpoint / resume on the GPU (cmbs_save_state / cmbs_load_state,
cosmomc_amd.checkpoint): a run stopped at a checkpoint and resumed in a fresh
sampler continues every chain exactly -- the same points, likelihoods,
multiplicities and accept counts, the same chain files and history -- as the
run that never stopped.  The reference (SampleCollector.f90:139-202,
GeneralSetup.f90:123-131) restarts from the last chain row with a new random
sequence, so there is no reference output to pin; the uninterrupted run is
the oracle here."""
import numpy as np
import pytest

from cosmomc_amd import synthetic as syn

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _gauss_sampler(ch, W):
    from cosmomc_amd.sampler import BatchedMCMC
    n = ch["n"]
    s = BatchedMCMC(W, n, list(range(1, n + 1)), ch["blocks"], ch["slow_block_max"], ch["pmin"], ch["pmax"],
                    ch["prior_mean"], ch["prior_std"], oversample_fast=ch["oversample_fast"],
                    propose_scale=ch["propose_scale"], temperature=ch["temperature"], seed_ij=ch["ij"],
                    seed_kl=ch["kl"])
    s.set_test_gaussian(np.array(ch["cov"]), np.array(ch["center"]))
    return s


def _same_state(a, b):
    for x, y in zip(a.state(), b.state()):
        np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("name", ["gauss6_blocked", "gauss6_fast_only", "gauss3_n1_blocks"])
def test_resume_continues_chains_exactly(rng_golden, tmp_path, name):
    from cosmomc_amd.checkpoint import read_checkpoint, write_checkpoint
    ch = rng_golden["chains"][name]
    W, fast = 128, bool(ch["fast_only"])
    a = _gauss_sampler(ch, W)
    a.set_covariance(np.array(ch["cov"]))
    a.set_start(np.tile(np.array(ch["P0"]), (W, 1)))
    a.step(25, fast_only=fast)
    root = str(tmp_path / "run")
    write_checkpoint(root, a, np.array(ch["cov"]), collector={"num_sample": 25})
    a.step(40, fast_only=fast)
    b = _gauss_sampler(ch, W)
    assert read_checkpoint(root, b) == {"num_sample": 25}
    b.step(40, fast_only=fast)
    _same_state(a, b)


def test_resume_dragging(rng_golden, tmp_path):
    from cosmomc_amd.checkpoint import read_checkpoint, write_checkpoint
    ch = rng_golden["chains"]["gauss6_drag"]
    W = 64
    a = _gauss_sampler(ch, W)
    a.set_covariance(np.array(ch["cov"]))
    a.set_start(np.tile(np.array(ch["P0"]), (W, 1)))
    a.step_drag(6, 3.0)
    root = str(tmp_path / "drag")
    write_checkpoint(root, a, np.array(ch["cov"]))
    a.step_drag(6, 3.0)
    b = _gauss_sampler(ch, W)
    read_checkpoint(root, b)
    b.step_drag(6, 3.0)
    _same_state(a, b)


def test_resume_plik_chain_files_and_history(tmp_path):
    """plik_lite fast chains with chain files and the history ring: the run
    that crashed after its checkpoint (rows already written past it) and was
    resumed writes byte-identical chain files to the uninterrupted run, and
    the convergence window statistics agree."""
    from cosmomc_amd.chains import ChainWriter
    from cosmomc_amd.checkpoint import read_checkpoint, write_checkpoint
    from cosmomc_amd.converge import ConvergenceExchange
    from cosmomc_amd.likelihood import NativeCMBLikelihood
    from cosmomc_amd.sampler import BatchedMCMC
    data = syn.make_plik_lite(12345)
    like = NativeCMBLikelihood("PLIK_LITE", data.write(str(tmp_path)))
    like.nuisance_indices = [2]
    W = 96
    dl = torch.tensor(syn.walker_theory(W, seed=3, n_fields=3), device="cuda")
    P0 = np.array([0.0222, 1.0, 3.05])
    cov = np.array([[0.002 ** 2]])

    def sampler():
        s = BatchedMCMC(W, 3, [2], [[1]], 0, [0.0222, 0.9, 3.05], [0.0222, 1.1, 3.05], [0.0, 1.0, 0.0],
                        [0.0, 0.0025, 0.0], seed_ij=55, seed_kl=66)
        s.add_likelihood(like, dl)
        s.enable_history(50)
        return s

    ref = sampler()
    ref.set_covariance(cov)
    ref.set_start(np.tile(P0, (W, 1)))
    cw = ChainWriter(str(tmp_path / "ref"), ["calPlanck"], likelihoods=[like.description()])
    for _ in range(3):
        ref.step(30, fast_only=True)
        cw.append(ref)
    cw.close()

    a = sampler()
    a.set_covariance(cov)
    a.set_start(np.tile(P0, (W, 1)))
    ex = ConvergenceExchange(1)
    ex.flukecheck = True
    cwa = ChainWriter(str(tmp_path / "run"), ["calPlanck"], likelihoods=[like.description()])
    for _ in range(2):
        a.step(30, fast_only=True)
        cwa.append(a)
    write_checkpoint(str(tmp_path / "run"), a, cov, chains=cwa, exchange=ex)
    a.step(30, fast_only=True)
    cwa.append(a)                                   # written, then the job dies
    del a, cwa

    b = sampler()
    ex2 = ConvergenceExchange(1)
    cwb = ChainWriter(str(tmp_path / "run"), ["calPlanck"], likelihoods=[like.description()])
    read_checkpoint(str(tmp_path / "run"), b, chains=cwb, exchange=ex2)
    assert ex2.flukecheck
    assert b.history_count() == 60
    b.step(30, fast_only=True)
    cwb.append(b)
    cwb.close()
    _same_state(ref, b)
    for w in range(W):
        assert (tmp_path / f"run_{w + 1}.txt").read_bytes() == (tmp_path / f"ref_{w + 1}.txt").read_bytes()
    for x, y in zip(ref.history_stats(45, 89), b.history_stats(45, 89)):
        assert torch.equal(x, y)


def test_resume_two_likelihoods(cmbl_golden, refdata, tmp_path):
    """plik_lite + Planck 2018 lensing sharing calPlanck: the image carries
    both likelihoods' current terms, and the resumed run (chains and history
    terms) matches the uninterrupted one."""
    import os
    from cosmomc_amd.checkpoint import read_checkpoint, write_checkpoint
    from cosmomc_amd.likelihood import NativeCMBLikelihood
    from cosmomc_amd.sampler import BatchedMCMC
    lc = cmbl_golden["cases"]["lensing_consext8"]
    plik = NativeCMBLikelihood("PLIK_LITE", syn.make_plik_lite(12345).write(str(tmp_path)))
    lens = NativeCMBLikelihood(lc["tag"], os.path.join(refdata, lc["dataset"]), lc["overrides"])
    plik.nuisance_indices = lens.nuisance_indices = [2]
    W = 64
    dl = torch.tensor(syn.walker_theory(W, seed=5, n_fields=10, ld_field=2512), device="cuda")
    cov = np.array([[0.002 ** 2]])

    def sampler():
        s = BatchedMCMC(W, 3, [2], [[1]], 0, [0.0222, 0.9, 3.05], [0.0222, 1.1, 3.05], [0.0, 1.0, 0.0],
                        [0.0, 0.0025, 0.0], seed_ij=77, seed_kl=88)
        s.add_likelihood(plik, dl)
        s.add_likelihood(lens, dl)
        s.enable_history(40)
        return s

    a = sampler()
    a.set_covariance(cov)
    a.set_start(np.tile([0.0222, 1.0, 3.05], (W, 1)))
    a.step(15, fast_only=True)
    write_checkpoint(str(tmp_path / "two"), a, cov)
    a.step(15, fast_only=True)
    b = sampler()
    read_checkpoint(str(tmp_path / "two"), b)
    b.step(15, fast_only=True)
    _same_state(a, b)
    np.testing.assert_array_equal(a.history_terms(25, 5), b.history_terms(25, 5))
    assert a.history_terms(29, 1).shape == (1, 2, W)


def test_checkpoint_before_first_step(rng_golden, tmp_path):
    """A checkpoint written right after set_start (empty history, no chain
    rows yet) resumes: the history ring, chain files and chains continue as in
    the uninterrupted run; rows a crashed run wrote after the checkpoint are cut."""
    from cosmomc_amd.chains import ChainWriter
    from cosmomc_amd.checkpoint import read_checkpoint, write_checkpoint
    ch = rng_golden["chains"]["gauss6_blocked"]
    W = 64

    def sampler():
        s = _gauss_sampler(ch, W)
        s.enable_history(64)
        return s
    ref = sampler()
    ref.set_covariance(np.array(ch["cov"]))
    ref.set_start(np.tile(np.array(ch["P0"]), (W, 1)))
    cw = ChainWriter(str(tmp_path / "ref"), [f"p{i}" for i in range(6)])
    ref.step(30)
    cw.append(ref)
    cw.close()
    a = sampler()
    a.set_covariance(np.array(ch["cov"]))
    a.set_start(np.tile(np.array(ch["P0"]), (W, 1)))
    cwa = ChainWriter(str(tmp_path / "run"), [f"p{i}" for i in range(6)])
    root = str(tmp_path / "run")
    write_checkpoint(root, a, np.array(ch["cov"]), chains=cwa)
    a.step(20)
    cwa.append(a)                                     # the crashed run's rows
    b = sampler()
    cwb = ChainWriter(str(tmp_path / "run"), [f"p{i}" for i in range(6)])
    read_checkpoint(root, b, chains=cwb)
    assert b.history_count() == 0
    b.step(30)
    cwb.append(b)
    cwb.close()
    _same_state(ref, b)
    for w in range(W):
        assert (tmp_path / f"run_{w + 1}.txt").read_bytes() == (tmp_path / f"ref_{w + 1}.txt").read_bytes()


def test_resume_slow_steps_refreshes_theory(tmp_path):
    """Full GetNewSample steps with theory recomputed at trial points (slow
    amplitude A, theory = A x base): after a resume in a fresh sampler whose
    theory rows hold the base theory, stepping fails until refresh_theory has
    recomputed the theory at the restored points; then every chain continues
    exactly as in the uninterrupted run."""
    from cosmomc_amd._native import NativeError
    from cosmomc_amd.checkpoint import read_checkpoint, write_checkpoint
    from cosmomc_amd.likelihood import NativeCMBLikelihood
    from cosmomc_amd.sampler import BatchedMCMC
    data = syn.make_plik_lite(12345)
    like = NativeCMBLikelihood("PLIK_LITE", data.write(str(tmp_path)))
    like.nuisance_indices = [2]
    W = 64
    base = torch.tensor(syn.base_theory(2508)[:3], device="cuda")
    cov = np.diag([0.002 ** 2, 0.0025 ** 2])

    def sampler():
        s = BatchedMCMC(W, 2, [1, 2], [[1], [2]], 1, [0.9, 0.9], [1.1, 1.1], [0.0, 1.0], [0.0, 0.0025],
                        oversample_fast=2, seed_ij=81, seed_kl=82)
        theory = base.unsqueeze(0).repeat(W, 1, 1).contiguous()
        trial = torch.empty_like(theory)
        s.add_likelihood(like, theory)
        s.set_trial_theory(0, trial)
        s.set_covariance(cov)

        def theory_fn(P):
            trial.copy_(base.unsqueeze(0) * P[0].reshape(-1, 1, 1))
        return s, theory, theory_fn
    a, th_a, fn_a = sampler()
    a.set_start(np.tile([1.0, 1.0], (W, 1)))
    a.step_theory(20, theory_fn=fn_a)
    root = str(tmp_path / "slow")
    write_checkpoint(root, a, cov)
    a.step_theory(20, theory_fn=fn_a)
    b, th_b, fn_b = sampler()
    read_checkpoint(root, b)
    with pytest.raises(NativeError, match="refresh"):
        b.step_theory(1, theory_fn=fn_b)
    b.refresh_theory(fn_b)
    b.step_theory(20, theory_fn=fn_b)
    _same_state(a, b)
    assert torch.equal(th_a, th_b)


def test_resume_with_chain_collector(tmp_path):
    """A run with the convergence collector (ChainCollector: per-walker
    Samples lists on device, walker-0 triggers, burn-in and update frequency
    on the host) checkpointed between exchanges and resumed in a fresh
    sampler + collector makes the same exchanges -- same R-1 and proposal
    covariance, same collector lists -- as the run that never stopped."""
    from cosmomc_amd.checkpoint import read_checkpoint, write_checkpoint
    from cosmomc_amd.converge import ChainCollector, CollectorSettings
    from cosmomc_amd.sampler import BatchedMCMC
    n, W, cap = 3, 96, 4000
    rng = np.random.default_rng(8)
    A = rng.standard_normal((n, n))
    cov = A @ A.T / n + np.eye(n)
    start = rng.standard_normal((W, n))

    def make():
        s = BatchedMCMC(W, n, [1, 2, 3], [[1, 2], [3]], 1, -30 * np.ones(n), 30 * np.ones(n), seed_ij=71,
                        seed_kl=72)
        s.set_covariance(cov)
        s.set_test_gaussian(cov, np.zeros(n))
        s.enable_history(cap)
        c = ChainCollector(s, CollectorSettings(MPI_R_Stop=0.01, covariance_is_diagonal=True), num_slow=2,
                           num_fast=1, sample_capacity=cap)
        return s, c

    def run(s, c, blocks, out, prop):
        for _ in range(blocks):
            s.step(c.next_block())
            r = c.process()
            if r is not None:
                out.append((r.R, r.propose_cov.copy()))
                if r.update_proposal:
                    s.set_covariance(r.propose_cov)
                    prop = r.propose_cov
        return prop

    a, ca = make()
    a.set_start(start)
    full = []
    run(a, ca, 60, full, cov)
    assert len(full) >= 4, "too few exchanges for the test to mean much"

    b, cb = make()
    b.set_start(start)
    part = []
    prop = run(b, cb, 25, part, cov)
    assert 0 < len(part) < len(full)
    root = str(tmp_path / "coll")
    write_checkpoint(root, b, prop, chain_collector=cb)        # with the proposal in force
    c_, cc = make()                               # fresh sampler and collector, as a restarted job
    read_checkpoint(root, c_, chain_collector=cc)
    run(c_, cc, 35, part, prop)
    assert len(part) == len(full)
    for (r1, p1), (r2, p2) in zip(full, part):
        assert r1 == r2
        np.testing.assert_array_equal(p1, p2)
    for x, y in zip(a.collector_state(), c_.collector_state()):
        np.testing.assert_array_equal(x, y)
    _same_state(a, c_)
