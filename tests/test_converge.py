"""Convergence exchange (TMpiChainCollector_UpdateCovAndCheckConverge,
SampleCollector.f90:212-322; GelmanRubinEvalues, samples.f90:41-67).

CPU: the C oracle and the host eigen-step against the compiled reference's
GelmanRubinEvalues (tests/golden/gr_ref.json), and the multi-rank exchange
(gloo, world size 2 and 3) against the single-process pooled statistics.
"""
import os
import socket

import numpy as np
import pytest

import pyoracle as po
from cosmomc_amd import synthetic as syn
from cosmomc_amd.converge import ConvergenceExchange, CollectorSettings, gelman_rubin_evalues, reference_window

torch = pytest.importorskip("torch")


class HostMoments:
    """Host restatement of cmbs_chain_moments' partial-sum layout for a set of
    chains held in numpy (the device kernel is covered by the GPU tests)."""
    device = "cpu"

    def __init__(self, chains):
        self.x = chains                      # [M, T, n]

    def chain_moments(self, first, last, gmean=None):
        rows = self.x[:, first:last + 1]
        cnt = rows.shape[1]
        m = rows.mean(axis=1)
        d = rows - m[:, None, :]
        C = np.einsum("mti,mtj->mij", d, d) / cnt
        n = m.shape[1]
        if gmean is not None:
            g = np.asarray(gmean)
            dm = m - g
            out = (cnt * np.einsum("mi,mj->ij", dm, dm)).ravel()
        else:
            out = np.concatenate([[cnt * len(m)], cnt * m.sum(0), (cnt * C.sum(0)).ravel(), C.sum(0).ravel(),
                                  [len(m)]])
        return torch.tensor(out, dtype=torch.float64)


@pytest.mark.parametrize("case", ["gr_n3_m8", "gr_n6_m16", "gr_n2_m4", "gr_n7_m32"])
def test_oracle_gelman_rubin_vs_reference(gr_golden, case):
    c = gr_golden[case]
    R = po.gelman_rubin(np.array(c["cov"]), np.array(c["meanscov"]))
    assert R == pytest.approx(c["R"], rel=1e-10)


@pytest.mark.parametrize("case", ["gr_n3_m8", "gr_n6_m16", "gr_n2_m4", "gr_n7_m32"])
def test_host_evalues_vs_reference(gr_golden, case):
    c = gr_golden[case]
    ok, ev = gelman_rubin_evalues(np.array(c["cov"]), np.array(c["meanscov"]))
    assert ok
    np.testing.assert_allclose(np.sort(ev), np.sort(c["evals"]), rtol=1e-9, atol=1e-14)


@pytest.mark.parametrize("case", ["gr_n3_m8", "gr_n7_m32"])
def test_single_rank_exchange_matches_pooled(gr_golden, case):
    c = gr_golden[case]
    x = syn.chain_ensemble(c["chains"], c["samples"], c["n"], c["seed"], c["spread"])
    first, last = reference_window(c["samples"])
    ex = ConvergenceExchange(c["n"], CollectorSettings(MPI_Min_Sample_Update=50))
    r = ex.update_cov_and_check_converge(HostMoments(x), first, last)
    assert r.n_chains == c["chains"]
    np.testing.assert_allclose(r.mean, c["mean"], rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(r.propose_cov, c["propose_cov"], rtol=1e-11, atol=1e-15)
    np.testing.assert_allclose(r.cov, c["cov"], rtol=1e-11, atol=1e-15)
    np.testing.assert_allclose(r.meanscov, c["meanscov"], rtol=1e-9, atol=1e-15)
    assert r.R == pytest.approx(c["R"], rel=1e-9)
    assert r.enough_samples and r.update_proposal == (r.R < 2.0)


def test_flukecheck_needs_two_passes():
    """ConvergeStatus(.true.) only on the second consecutive R < MPI_R_Stop."""
    x = syn.chain_ensemble(8, 400, 3, 9, 0.0)
    ex = ConvergenceExchange(3, CollectorSettings(MPI_R_Stop=0.5, MPI_Min_Sample_Update=50))
    first, last = reference_window(400)
    r1 = ex.update_cov_and_check_converge(HostMoments(x), first, last)
    r2 = ex.update_cov_and_check_converge(HostMoments(x), first, last)
    assert r1.R < 0.5 and not r1.converged and r2.converged


def test_not_enough_samples():
    x = syn.chain_ensemble(4, 40, 2, 3, 0.1)
    ex = ConvergenceExchange(2)                       # MPI_Min_Sample_Update = 200
    r = ex.update_cov_and_check_converge(HostMoments(x), *reference_window(40))
    assert not r.enough_samples and not r.update_proposal and not r.converged


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, case, q):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        x = syn.chain_ensemble(case["chains"], case["samples"], case["n"], case["seed"], case["spread"])
        parts = np.array_split(np.arange(case["chains"]), world)      # contiguous walker ranges per GPU
        ex = ConvergenceExchange(case["n"], CollectorSettings(MPI_Min_Sample_Update=50))
        r = ex.update_cov_and_check_converge(HostMoments(x[parts[rank]]), *reference_window(case["samples"]))
        q.put((rank, r.R, r.propose_cov.tolist(), r.meanscov.tolist(), r.n_chains))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_multirank_exchange_gloo(gr_golden, world):
    import torch.multiprocessing as mp
    case = gr_golden["gr_n6_m16"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, R, pc, mc, M in res:
        assert M == case["chains"]
        assert R == pytest.approx(case["R"], rel=1e-9)
        np.testing.assert_allclose(pc, case["propose_cov"], rtol=1e-11, atol=1e-15)
        np.testing.assert_allclose(mc, case["meanscov"], rtol=1e-9, atol=1e-15)


def test_confid_val_restatement_vs_reference():
    """pyoracle.confid_val == the compiled TSampleList%ConfidVal (samples.f90:70-110)."""
    import pyoracle as po
    from conftest import load_golden
    from cosmomc_amd import synthetic as syn
    g = load_golden("confid_ref.json")
    for name, c in g.items():
        v = syn.gaussians(c["seed"], c["samples"] * c["columns"]).reshape(c["samples"], c["columns"])
        if c["ties"]:
            v = np.round(v * 3) / 3
        for j in range(c["columns"]):
            lo, hi = po.confid_val(v[:, j], c["limfrac"], c["ix1"], c["ix2"])
            assert lo == pytest.approx(c["limits"][j][0], rel=1e-14, abs=1e-15), name
            assert hi == pytest.approx(c["limits"][j][1], rel=1e-14, abs=1e-15), name


def _collector_run(W_total, world, rank, q):
    """ChainCollector over FakeCollectorSampler walkers [rank*W, (rank+1)*W):
    returns the (history step, R, Count of walker 0) of every exchange."""
    from collector_fake import FakeCollectorSampler
    from cosmomc_amd.converge import ChainCollector, CollectorSettings
    W = W_total // world
    s = FakeCollectorSampler(W, first_walker=rank * W)
    st = CollectorSettings(MPI_R_Stop=0.02, MPI_Sample_update_freq=5, MPI_Check_Limit_Converge=True,
                           MPI_Limit_Converge_Err=0.5)
    col = ChainCollector(s, st, num_slow=2, num_fast=1, sample_capacity=100000)
    log = []
    while s.history_count() < 1500 and not col.done:
        s.step(col.next_block())
        r = col.process()
        if r is not None:
            log.append((s.history_count(), r.R, col.count0, bool(r.converged)))
    q.put((rank, log, col.burn0, col.update_freq))


def _collector_rank(rank, world, port, W_total, q):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        _collector_run(W_total, world, rank, q)
    finally:
        dist.destroy_process_group()


def test_chain_collector_two_ranks_match_one(tmp_path):
    """ChainCollector sharded over 2 gloo ranks (all_burn and the minimum
    count as all-reduces, walker 0 on rank 0 triggering) exchanges at the same
    steps with the same R-1 as one rank holding every walker; burn-in scales
    the update frequency by num_params_used; CheckLimitsConverge ends the run."""
    import queue as _q
    import torch.multiprocessing as mp
    W_total = 16
    q1 = _q.Queue()
    _collector_run(W_total, 1, 0, q1)
    _, ref_log, burn0, freq = q1.get()
    assert burn0 and freq == 15 and len(ref_log) > 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_collector_rank, args=(r, 2, port, W_total, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, log, _, _ in res:
        assert [x[0] for x in log] == [x[0] for x in ref_log]
        assert [x[2] for x in log] == [x[2] for x in ref_log]
        np.testing.assert_allclose([x[1] for x in log], [x[1] for x in ref_log], rtol=1e-9)
        assert [x[3] for x in log] == [x[3] for x in ref_log]
