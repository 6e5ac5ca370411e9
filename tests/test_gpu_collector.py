"""Sample collector on the GPU (cmbs_collector_*, cosmomc_amd.converge.ChainCollector)
against the item-by-item restatement of TMpiChainCollector_AddNewPoint
(oracle/pyoracle.py collector_samples, SampleCollector.f90:324-397), the
pooled statistics (pool_chain_statistics, :233-286) and ConfidVal
(confid_val, pinned to the compiled samples.f90 in tests/test_converge.py)."""
import numpy as np
import pytest

import pyoracle as po

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _gauss(W, n=3, seed=5, cap=900):
    from cosmomc_amd.sampler import BatchedMCMC
    rng = np.random.default_rng(seed)
    A = rng.standard_normal((n, n))
    cov = A @ A.T / n + np.eye(n)
    used = list(range(1, n + 1))
    s = BatchedMCMC(W, n, used, [used[:2], used[2:]], 1, -30 * np.ones(n), 30 * np.ones(n), seed_ij=41 + seed,
                    seed_kl=43)
    s.set_covariance(cov)
    s.set_test_gaussian(cov, np.zeros(n))
    s.set_start(rng.standard_normal((W, n)))
    s.enable_history(cap)
    return s


def _restate(s, steps_all, min_update, thin=1):
    """Per-walker restated Samples lists over the sampler's whole history."""
    T = s.history_count()
    rows = s.history_host(0, T)                     # [T, n + 1, W]
    out = []
    for w in range(s.W):
        st = po.collector_samples(rows[:, :, w], steps_all, min_update, True, thin)
        out.append(st)
    return rows, out


@pytest.mark.parametrize("output_thin", [1, 2])
def test_samples_lists_burn_and_window_moments(output_thin):
    """Blocks of steps added as they are recorded: every walker's list
    (count, burn flag) equals the restatement's, and the device window
    moments equal the reference pooling over the restated lists."""
    W, min_update = 70, 60
    s = _gauss(W)
    s.collector_enable(900)
    added = []
    for blk in (37, 100, 1, 150, 212, 200):
        first = s.history_count()
        s.step(blk)
        steps = [t for t in range(first, s.history_count()) if (t + 1) % output_thin == 0]
        s.collector_add(steps, min_update)
        added += steps
    rows, ref = _restate(s, added, min_update)
    start, count, burn, thin = s.collector_state()
    assert np.all(thin == 1)
    np.testing.assert_array_equal(count, [len(r["items"]) for r in ref])
    np.testing.assert_array_equal(burn, [int(r["burn"]) for r in ref])
    assert burn.sum() > W // 2, "too few walkers burned in for the test to mean much"
    n = 3
    samples = [rows[r["items"], :n, w] for w, r in enumerate(ref)]
    pooled = po.pool_chain_statistics(samples)
    p1 = s.collector_moments().cpu().numpy()
    norm = p1[0]
    assert norm == pytest.approx(pooled["counts"].sum())
    np.testing.assert_allclose(p1[1:1 + n] / norm, pooled["mean"], rtol=1e-11, atol=1e-13)
    np.testing.assert_allclose(p1[1 + n:1 + n + n * n].reshape(n, n) / norm, pooled["propose_cov"], rtol=1e-10,
                               atol=1e-13)
    M = int(round(p1[-1]))
    np.testing.assert_allclose(p1[1 + n + n * n:1 + n + 2 * n * n].reshape(n, n) / M, pooled["cov"], rtol=1e-10,
                               atol=1e-13)
    p2 = s.collector_moments(p1[1:1 + n] / norm).cpu().numpy()
    np.testing.assert_allclose(p2.reshape(n, n) / norm * M / (M - 1), pooled["meanscov"], rtol=1e-8, atol=1e-13)


def test_limits_and_thin():
    """ConfidVal limits of every walker's window (radix select on device) equal
    the sorted restatement; Samples%Thin(2) keeps items 1, 3, 5, ... of the
    walkers above the limit and doubles their MPI_thin_fac."""
    W, min_update = 66, 40
    s = _gauss(W, seed=9, cap=700)
    s.collector_enable(700)
    s.step(650)
    steps = list(range(650))
    s.collector_add(steps, min_update)
    rows, ref = _restate(s, steps, min_update)
    for frac in (0.025, 0.3):
        lim = s.collector_limits([0, 2], frac).cpu().numpy()
        for w in (0, 1, 37, 65):
            items = ref[w]["items"]
            cnt = len(items)
            for c, j in enumerate((0, 2)):
                lo, hi = po.confid_val(rows[items, j, w], frac, cnt // 2, cnt)
                assert lim[w, c, 0] == pytest.approx(lo, rel=1e-15, abs=1e-300), (w, j, frac)
                assert lim[w, c, 1] == pytest.approx(hi, rel=1e-15, abs=1e-300), (w, j, frac)
    _, count, _, _ = s.collector_state()
    limit = int(np.median(count))
    s.collector_thin(limit)
    _, count2, _, thin = s.collector_state()
    for w in range(W):
        c = int(count[w])
        if c > limit:
            assert count2[w] == (c - 1) // 2 + 1 and thin[w] == 2
            ref[w]["items"] = ref[w]["items"][::2]
        else:
            assert count2[w] == c and thin[w] == 1
    # after thinning only every second sample_num is kept (MPI_thin_fac 2)
    first = s.history_count()
    s.step(40)
    new = list(range(first, s.history_count()))
    s.collector_add(new, min_update)
    T = s.history_count()
    rows = s.history_host(0, T)
    _, count3, _, _ = s.collector_state()
    for w in range(W):
        st = dict(ref[w])
        st["items"] = list(st["items"])
        po.collector_samples(rows[:, :, w], new, min_update, True, int(thin[w]), st)
        assert count3[w] == len(st["items"]), w


def test_chain_collector_drives_exchange(tmp_path):
    """ChainCollector: walker 0's burn scales the update frequency by
    num_params_used and sets MPI_Min_Sample_Update = 50 + 4 num_slow + 5 num_fast;
    exchanges happen exactly when walker 0's Count is a multiple of the
    frequency; the run converges and writes root.converge_stat."""
    from cosmomc_amd.converge import ChainCollector, CollectorSettings
    W = 96
    s = _gauss(W, seed=3, cap=6000)
    st = CollectorSettings(MPI_R_Stop=0.05, MPI_Sample_update_freq=10)
    col = ChainCollector(s, st, num_slow=2, num_fast=1, root=str(tmp_path / "run"))
    assert col.min_after_burn == 50 + 8 + 1 + 4
    trig = []
    while s.history_count() + col.next_block() <= 6000 and not col.done:
        s.step(col.next_block())
        r = col.process()
        if r is not None:
            trig.append(col.count0)
            if r.update_proposal:
                s.set_covariance(r.propose_cov)
    assert col.burn0 and col.all_burn and col.update_freq == 30
    # the first exchange may wait for the last walkers to reach Min + 1 samples (Waiting, :431-434)
    assert len(trig) > 1 and all(c % 30 == 0 for c in trig[1:])
    assert col.done, [r.R for r in col.results][-5:]
    assert open(tmp_path / "run.converge_stat").read().splitlines()[-1] == "Done"
