#!/usr/bin/env python3
"""Headline benchmark: fast-parameter likelihood evals/s on plik_lite TTTEEE.

One *step* = one fast-parameter Metropolis step of every walker on this GPU
(reference TMetropolisSampler FastParameterSample, source/MCMC.f90:309-335):
BlockedProposer GetProposalFast (propose.f90:283-289) -> native plik_lite
-lnL on the walker's cached slow-parameter theory (CMB.f90:305-329, full
binning + 613x613 quadratic form every step, as the reference) + calPlanck
prior -> Metropolis accept.  Each step is W likelihood evaluations.

Workload: BASELINE.json configs[2] -- plik_lite_TTTEEE + Planck 2018 lensing
(the reference's own consext8 dataset, tests/golden/refdata.tar.xz), 1024
walkers on one MI355X, cached slow block -- without its lowl term (clik
commander: library unavailable, parity-unpinned).  Each evaluation is both
likelihoods + the calPlanck prior.  Synthetic theory of the Planck l_max shape
(cosmomc_amd.synthetic).  Multi-GPU: walkers are sharded across ranks with no
per-step collective ("weak" scaling).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--walkers 1024] [--no-lensing]

The JSON line also carries, outside the headline value: "convergence" (R-1 vs
wall-clock for the headline workload), "config1_tt" (BASELINE configs[1]:
plik_lite TT on the reference's fixed best-fit theory, 256 walkers per GPU),
"config4_fast21" (BASELINE configs[3]
as a sampler-throughput workload: 21 fast parameters, 512 walkers per GPU;
full plik needs the absent clik), "config5_bk15_plik" (BASELINE
configs[4]: BK15 + plik_lite jointly, fast-step throughput and R-1 vs
wall-clock with the cross-GPU exchange) and "config2_drag" (BASELINE
configs[2] with its fast/slow dragging: a slow amplitude whose theory comes
from a theory function at every drag, plik_lite + lensing at 1024 walkers).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "fast-param likelihood evals/sec/node (plik_lite_TTTEEE ℓmax=2508); R-1 vs wall-clock"
N_B = 613            # plik_lite TTTEEE bins (CMB.f90:35)
N_L = 2479 + 1967 + 1967   # l values binned per eval (TT 30..2508, TE/EE 30..1996)
FLOPS_QUADFORM = 2 * N_B * N_B + 2 * N_B          # DSYMV + DDOT per eval
FLOPS_EVAL = 2 * N_L + 2 * N_B * N_B + 4 * N_B    # 766,816
BYTES_BIN = 8 * N_L + 8                            # D_l + cal per walker, read once
PEAK_FP64_TFLOPS = 78.6    # MI355X dense FP64 matrix, spec (datasheet)
PEAK_HBM_GBS = 8000.0      # MI355X HBM3E, MI355X_MICROARCH.md


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=500)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--walkers", type=int, default=1024, help="walkers per GPU")
    p.add_argument("--groups", type=int, default=int(os.environ.get("CMBS_GROUPS", "1")),
                   help="walker groups stepped on concurrent streams (cmbs_set_groups)")
    p.add_argument("--cpu-seconds", type=float, default=2.0, help="per-round CPU baseline sample (5 rounds)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-lensing", action="store_true", help="plik_lite only (configs[2] minus lensing)")
    p.add_argument("--cache-steps", type=int, default=200,
                   help="steps of the separately labelled binned-theory-cache leg (SURVEY 8(d)); -1 skips it")
    p.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) on the node; gloo to rehearse ranks")
    p.add_argument("--converge-seconds", type=float, default=20.0,
                   help="R-1 vs wall-clock run after the throughput timing (0 = skip)")
    p.add_argument("--config1-seconds", type=float, default=10.0,
                   help="plik_lite TT at 256 walkers (BASELINE configs[1]) throughput and R-1 run (< 0 = skip)")
    p.add_argument("--config4-seconds", type=float, default=30.0,
                   help="21-fast-parameter sampler workload (BASELINE configs[3]) throughput and R-1 run (< 0 = skip)")
    p.add_argument("--config5-seconds", type=float, default=60.0,
                   help="BK15 + plik_lite (BASELINE configs[4]) throughput and R-1 run (< 0 = skip)")
    p.add_argument("--drag-seconds", type=float, default=30.0,
                   help="configs[2] with fast/slow dragging: throughput and R-1 run (< 0 = skip)")
    return p.parse_args()


LENS_DATASET = "planck_lensing_2018/smicadx12_Dec5_ftl_mv2_ndclpp_p_teb_consext8.dataset"


def extract_refdata(tmpdir):
    """The reference's own lensing dataset files, from the committed fixture."""
    import io
    import lzma
    import tarfile
    d = os.path.join(tmpdir, "refdata")
    with open(os.path.join(ROOT, "tests", "golden", "refdata.tar.xz"), "rb") as f:
        tar = tarfile.open(fileobj=io.BytesIO(lzma.decompress(f.read())))
        try:
            tar.extractall(d, filter="data")
        except TypeError:
            tar.extractall(d)
    return d


def build_problem(W, rank, tmpdir, groups=1, lensing=True):
    import torch
    from cosmomc_amd import synthetic as syn
    from cosmomc_amd.likelihood import NativeCMBLikelihood
    from cosmomc_amd.sampler import BatchedMCMC
    data = syn.make_plik_lite(12345)
    ds = data.write(tmpdir)
    like = NativeCMBLikelihood("PLIK_LITE", ds)
    likes = [like]
    if lensing:
        lens = NativeCMBLikelihood("lensing", os.path.join(extract_refdata(tmpdir), LENS_DATASET))
        lens.nuisance_indices = [7]                   # calPlanck, shared with plik_lite
        likes.append(lens)
    # parameters: 6 slow cosmological parameters (fixed theory cached per walker)
    # + calPlanck (fast, nuisance of plik_lite); blocks slow | fast
    names = ["omegabh2", "omegach2", "theta", "tau", "logA", "ns"]
    P0 = np.array([0.02237, 0.1200, 1.04092, 0.0544, 3.044, 0.9649, 1.0])
    sig = np.array([0.00015, 0.0012, 0.00031, 0.0073, 0.014, 0.0042, 0.0025])
    pmin = P0 - 50 * sig
    pmax = P0 + 50 * sig
    pmin[6], pmax[6] = 0.9, 1.1                       # param[calPlanck]=1 0.9 1.1 ...
    pm = np.zeros(7)
    ps = np.zeros(7)
    pm[6], ps[6] = 1.0, 0.0025                        # prior[calPlanck]=1 0.0025
    like.nuisance_indices = [7]
    smp = BatchedMCMC(W, 7, list(range(1, 8)), [list(range(1, 7)), [7]], 1, pmin, pmax, pm, ps,
                      propose_scale=2.4, seed_ij=1802 + rank, seed_kl=9373, first_walker=rank * W)
    smp.set_covariance(np.diag(sig ** 2))
    smp.set_groups(groups)
    nf = 10 if lensing else 3
    theory = torch.tensor(syn.walker_theory(W, first_walker=rank * W, n_fields=nf, ld_field=2512), device="cuda")
    for lk in likes:
        smp.add_likelihood(lk, theory)
    smp.set_start(np.tile(P0, (W, 1)))
    return smp, likes, theory, names


def run_to_convergence(smp, num_slow, num_fast, seconds, world, cap, fast_only=True, stepper=None):
    """R-1 vs wall-clock with the reference's collector logic (ChainCollector:
    per-walker burn-in, all_burn, MPI_Min_Sample_Update = 50 + 4 num_slow +
    5 num_fast and update frequency 40 x num_params_used after burn-in,
    walker-0 triggered exchanges, SampleCollector.f90:324-460) and proposal
    learning, until R-1 < 0.01 twice running or `seconds` pass.  Every rank
    steps the same blocks (ChainCollector.next_block is rank-agreed)."""
    import torch
    from cosmomc_amd.converge import ChainCollector, CollectorSettings
    smp.enable_history(cap)
    col = ChainCollector(smp, CollectorSettings(MPI_R_Stop=0.01, covariance_is_diagonal=True), num_slow=num_slow,
                         num_fast=num_fast, sample_capacity=cap)
    trace, t0, done_at = [], time.perf_counter(), None
    while smp.history_count() + col.next_block() <= cap:
        if stepper is None:
            smp.step(col.next_block(), fast_only=fast_only)
        else:
            stepper(col.next_block())
        r = col.process()
        el = time.perf_counter() - t0
        if r is not None:
            trace.append([round(el, 4), smp.history_count(), r.R])
            if r.update_proposal:
                smp.set_covariance(r.propose_cov)
            if r.converged:
                done_at = el
                break
        stop = el > seconds
        if world > 1:
            import torch.distributed as dist
            flag = torch.tensor([1.0 if stop else 0.0], dtype=torch.float64, device="cuda")
            dist.all_reduce(flag, op=dist.ReduceOp.MAX)
            stop = flag.item() > 0
        if stop:
            break
    import torch.distributed as dist
    backend = dist.get_backend() if world > 1 else None
    return {"target_r_minus_1": 0.01, "min_sample_update": col.min_update, "update_freq": col.update_freq,
            "converged_wall_s": done_at, "trace_wall_s_steps_R": trace, "ranks": world,
            "exchanges": len(col.results),
            "exchange": (f"2 all_reduce per exchange over {backend} across {world} ranks "
                         "(SampleCollector.f90:248-251 MPI_ALLGATHER)") if world > 1 else "single rank, no collective"}


def convergence_run(W, rank, world, tmpdir, seconds, lensing=True):
    """R-1 vs wall-clock (the metric's second half): every walker samples the
    same posterior -- one shared cached slow point (theory stride 0), calPlanck
    fast, plik_lite (+ lensing) + the calPlanck prior -- from an overdispersed
    start; the collector's exchanges (ChainCollector: all_reduce over RCCL)
    learn the proposal until R-1 < 0.01 twice in a row
    (SampleCollector.f90:289-299) or time out."""
    import torch
    from cosmomc_amd import synthetic as syn
    from cosmomc_amd.likelihood import NativeCMBLikelihood
    from cosmomc_amd.sampler import BatchedMCMC
    likes = [NativeCMBLikelihood("PLIK_LITE", syn.make_plik_lite(12345).write(tmpdir))]
    if lensing:
        likes.append(NativeCMBLikelihood("lensing", os.path.join(extract_refdata(tmpdir), LENS_DATASET)))
    for lk in likes:
        lk.nuisance_indices = [7]
    P0 = np.array([0.02237, 0.1200, 1.04092, 0.0544, 3.044, 0.9649, 1.0])
    pmin, pmax = P0.copy(), P0.copy()
    pmin[6], pmax[6] = 0.9, 1.1
    pm, ps = np.zeros(7), np.zeros(7)
    pm[6], ps[6] = 1.0, 0.0025
    smp = BatchedMCMC(W, 7, [7], [[1]], 0, pmin, pmax, pm, ps, propose_scale=2.4, seed_ij=2002 + rank,
                      seed_kl=9373, first_walker=rank * W)
    smp.set_covariance(np.array([[0.0025 ** 2]]))
    th = torch.tensor(syn.walker_theory(1, n_fields=10 if lensing else 3, ld_field=2512), device="cuda")
    th = th.expand(W, th.shape[1], th.shape[2])       # ld_walker = 0: one slow point for everyone
    for lk in likes:
        smp.add_likelihood(lk, th)
    start = np.tile(P0, (W, 1))
    start[:, 6] = 1.0 + 0.01 * syn.gaussians(77 + rank, W)
    smp.set_start(start)
    out = run_to_convergence(smp, 0, 1, seconds, world, 20000)
    out.update({"workload": "plik_lite_TTTEEE" + (" + lensing" if lensing else "") + " on one shared slow point, "
                            "calPlanck fast, overdispersed start (1 +- 0.01)", "walkers_total": W * world})
    return out


KERNELS = ("plik_bin_delta", "plik_quadform_ksplit", "plik_quadform_corun", "mh_kernel", "rot_kernel",
           "cmbl_bk_prologue", "cmbl_window_kernel", "cmbl_reduce_kernel", "cmbl_hl_kernel", "cmbl_quadform",
           "cmbl_gauss_small_kernel", "theory_window_kernel", "drag_kernel", "plik_quadform_pair", "mh_step_first",
           "mh_step_kernel", "mh_step_last", "mh_bin_kernel")


def kernel_profile(smp, steps, stepper=None, per_step=False):
    """Average device time (us) per launch of every library kernel over `steps`
    more steps (HIP events on the launch stream); per_step: also the total per
    step of each kernel (its launches per step x its average)."""
    import torch
    from cosmomc_amd import _native as N
    N.profile_reset()
    N.profile_enable(True)
    if stepper:
        stepper(steps)
    else:
        smp.step(steps, fast_only=True)
    torch.cuda.synchronize()
    N.profile_enable(False)
    out, tot = {}, {}
    for k in KERNELS:
        ms, cnt = N.profile_read(k)
        if cnt:
            out[k] = round(ms / cnt * 1e3, 2)
            tot[k] = round(ms / steps * 1e3, 2)
    return (out, tot) if per_step else out


def drag_run(W, rank, world, tmpdir, seconds, steps=20, dragging_steps=3.0):
    """BASELINE configs[2] with its fast/slow dragging (MCMC.f90:357-420):
    plik_lite TTTEEE + Planck 2018 lensing on per-walker theory rows, one slow
    parameter (an amplitude A: theory = A x base D_l, computed by a theory
    function -- the CAMB stand-in -- at every drag's end point) and calPlanck
    fast; each drag interpolates over round(dragging_steps x num_fast) + 1
    points, evaluating both likelihoods at the start and end theories
    (1 + 2 x (interp - 1) evaluations per walker and drag).  Reports drag steps
    and likelihood evaluations per second and, when seconds > 0, R-1 vs
    wall-clock of A and calPlanck from an overdispersed start."""
    import torch
    from cosmomc_amd import synthetic as syn
    from cosmomc_amd.likelihood import NativeCMBLikelihood
    from cosmomc_amd.sampler import BatchedMCMC
    plik = NativeCMBLikelihood("PLIK_LITE", syn.make_plik_lite(12345).write(os.path.join(tmpdir, "c2p")))
    lens = NativeCMBLikelihood("lensing", os.path.join(extract_refdata(tmpdir), LENS_DATASET))
    plik.nuisance_indices = [2]
    lens.nuisance_indices = [2]
    base = torch.tensor(syn.walker_theory(1, n_fields=10, ld_field=2512), device="cuda")[0]
    pmin, pmax = np.array([0.95, 0.9]), np.array([1.05, 1.1])
    pm, ps = np.array([0.0, 1.0]), np.array([0.0, 0.0025])
    smp = BatchedMCMC(W, 2, [1, 2], [[1], [2]], 1, pmin, pmax, pm, ps, propose_scale=2.4, seed_ij=3003 + rank,
                      seed_kl=9373, first_walker=rank * W)
    smp.set_covariance(np.diag([0.002 ** 2, 0.0025 ** 2]))
    g = syn.gaussians(55 + rank, 2 * W).reshape(2, W)
    A0 = 1.0 + 0.005 * g[0]
    theory = (base.unsqueeze(0) * torch.tensor(A0, device="cuda").reshape(-1, 1, 1)).contiguous()
    end = torch.empty_like(theory)
    for lk in (plik, lens):
        smp.add_likelihood(lk, theory)
    smp.set_drag_theory(0, end)
    smp.set_drag_theory(1, end)
    smp.set_start(np.stack([A0, 1.0 + 0.005 * g[1]], axis=1))

    def theory_fn(P_end):                              # the drag's end-point theory (CAMB's place)
        torch.mul(base.unsqueeze(0), P_end[0].reshape(-1, 1, 1), out=end)

    def stepper(n):
        smp.step_drag(n, dragging_steps, theory_fn=theory_fn)
    stepper(2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stepper(steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    interp = max(2, int(round(dragging_steps * 1)) + 1)
    evals = 1 + 2 * (interp - 1)
    out = {"workload": "plik_lite_TTTEEE + Planck2018 lensing, per-walker theory rows, slow amplitude A dragged "
                       "(theory = A x base from a theory function at every drag) with calPlanck fast, "
                       f"dragging_steps={dragging_steps:g}",
           "walkers_total": W * world, "drag_steps_per_s": W * world * steps / dt,
           "likelihood_evals_per_s": W * world * steps * evals / dt, "evals_per_drag": evals,
           "ms_per_drag_step": dt / steps * 1e3}
    avg, tot = kernel_profile(smp, 5, stepper=stepper, per_step=True)
    out["avg_kernel_us"] = avg
    out["kernel_us_per_drag_step"] = tot
    if seconds > 0:
        out.update(run_to_convergence(smp, 1, 1, seconds, world, 40000, stepper=stepper))
    return out


N_B_TT = 215                                    # plik_lite TT bins
N_L_TT = 2479                                   # l = 30..2508
FLOPS_EVAL_TT = 2 * N_L_TT + 2 * N_B_TT * N_B_TT + 4 * N_B_TT   # 98,268 (SURVEY 8d with TT's sizes)
BYTES_BIN_TT = 8 * N_L_TT + 8


def binned_cache_run(smp, W, world, steps, warmup=20):
    """SURVEY 8(d)'s labelled variant, never the headline: the same sampler
    and workload with cmbs_set_binned_cache -- each walker's theory binned once
    per call (the theory is fixed within a fast-step call and the raw window
    sums are calibration-independent), so a step is plik's quadratic form, the
    lensing chi^2 and the Metropolis chain.  Roofline with the 2 N_l term
    dropped from F and the 8 N_l term from B, as 8(d) prescribes; the lensing
    likelihood's work is not counted."""
    import torch
    from cosmomc_amd import _native as N
    smp.set_binned_cache(True)
    smp.step(warmup, fast_only=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    smp.step(steps, fast_only=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    N.profile_reset()
    N.profile_enable(True)
    smp.step(steps, fast_only=True)
    torch.cuda.synchronize()
    N.profile_enable(False)
    tot, cnt = N.profile_read("mh_tail_kernel")
    smp.set_binned_cache(False)
    f_eval = 2 * N_B * N_B + 4 * N_B                                   # F without 2 N_l
    b_eval = 16 + (8 * N_B * N_B + 8 * 2479 + 8 * N_B) / W             # B without 8 N_l
    per_gpu = W * steps / dt
    ceil = min(PEAK_FP64_TFLOPS * 1e12, f_eval / b_eval * PEAK_HBM_GBS * 1e9)
    avg_us = tot / cnt * 1e3 if cnt else None
    qf = W * FLOPS_QUADFORM
    return {"label": "binned-theory cache (SURVEY 8(d) variant; NOT the headline): theory binned once per "
                     "cmbs_step call, every step runs plik's quadratic form + the lensing chi^2 + the chain",
            "walkers_total": W * world, "evals_per_s": W * world * steps / dt, "ms_per_step": dt / steps * 1e3,
            "step_roofline": {"achieved_tflops": per_gpu * f_eval / 1e12, "ceiling_tflops": ceil / 1e12,
                              "frac": per_gpu * f_eval / ceil,
                              "note": "per GPU: F = 2 N_b^2 + 4 N_b = 753,990 flop/eval, B = 16 + 3,030,888 / W "
                                      "bytes/eval (8(d) with the N_l terms dropped)"},
            "mh_tail_kernel": {"avg_launch_us": avg_us,
                               "mfma_frac": (qf / (avg_us * 1e-6) / 1e12 / PEAK_FP64_TFLOPS) if avg_us else None,
                               "note": "the quadratic form's 2 N_b^2 + 2 N_b flops per walker over the launch "
                                       "(chi^2 and chain in the same launch)"}}


def config1_run(W, rank, world, tmpdir, seconds, steps=300):
    """BASELINE configs[1]: plik_lite TT (batch2/plik_lite_TT.ini; the native
    TT path stands in for its clik file) on fixed CAMB C_l -- the reference's
    own base_plikHM best-fit theory_cl (tests/golden npz), one theory row for
    every walker (ld_walker = 0) -- with calPlanck fast and its prior
    (batch2/planck_calibration.ini), 256 walkers per GPU.  Fast-step
    throughput, the per-kernel times and the step's roofline with TT's F and B
    (F = 2 N_l + 2 N_b^2 + 4 N_b, B = 8 N_l + 8 per eval + C^-1
    once per launch), and, when seconds > 0, R-1 vs wall-clock from an
    overdispersed calPlanck start."""
    import torch
    from cosmomc_amd import synthetic as syn
    from cosmomc_amd.likelihood import NativeCMBLikelihood
    from cosmomc_amd.sampler import BatchedMCMC
    plik = NativeCMBLikelihood("PLIK_LITE", syn.make_plik_lite(12345).write(os.path.join(tmpdir, "c1p"), use_cl="TT"))
    plik.nuisance_indices = [1]
    smp = BatchedMCMC(W, 1, [1], [[1]], 0, [0.9], [1.1], [1.0], [0.0025], propose_scale=2.4, seed_ij=1101 + rank,
                      seed_kl=9373, first_walker=rank * W)
    smp.set_covariance(np.array([[0.0025 ** 2]]))
    base = syn.base_theory()[:3]
    th = torch.zeros((1, 3, 2512), dtype=torch.float64, device="cuda")
    th[0, :, :base.shape[1]] = torch.tensor(base, device="cuda")
    smp.add_likelihood(plik, th.expand(W, 3, 2512))
    smp.set_start((1.0 + 0.01 * syn.gaussians(11 + rank, W)).reshape(W, 1))
    smp.step(20, fast_only=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    smp.step(steps, fast_only=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    per_gpu = W * steps / dt
    ai = FLOPS_EVAL_TT / (BYTES_BIN_TT + 8 * N_B_TT * N_B_TT / W)
    ceil = min(PEAK_FP64_TFLOPS * 1e12, ai * PEAK_HBM_GBS * 1e9)
    out = {"workload": "plik_lite TT (215 bins, l 30..2508; batch2/plik_lite_TT.ini) on the reference's fixed "
                       "base_plikHM theory_cl, calPlanck fast + prior",
           "walkers_total": W * world, "evals_per_s": W * world * steps / dt, "ms_per_step": dt / steps * 1e3,
           "step_roofline": {"achieved_tflops": per_gpu * FLOPS_EVAL_TT / 1e12, "ceiling_tflops": ceil / 1e12,
                             "frac": per_gpu * FLOPS_EVAL_TT / ceil,
                             "note": "per GPU: F = 98,268 flop/eval, B = 19,840 + 369,800 / W bytes/eval"}}
    out["avg_kernel_us"], out["kernel_us_per_step"] = kernel_profile(smp, 100, per_step=True)
    if seconds > 0:
        out.update(run_to_convergence(smp, 0, 1, seconds, world, 20000))
    return out


def config4_run(W, rank, world, tmpdir, seconds, steps=200):
    """BASELINE configs[3] as a sampler-throughput workload:
    full plik's 21 fast foreground/calibration nuisances need clik, which is
    absent, so the likelihood is plik_lite TTTEEE (calPlanck) plus a correlated
    20-dimensional Gaussian over the other fast parameters (test_likelihood
    semantics, calclike.f90:180-199); one fast block of 21 parameters (random
    21-d rotations every 21 steps per walker), 512 walkers per GPU (4096 over 8),
    one shared cached slow point.  Reports fast-step throughput and, when
    seconds > 0, R-1 vs wall-clock with the exchange every 40 x 21 samples."""
    import torch
    from cosmomc_amd import synthetic as syn
    from cosmomc_amd.likelihood import NativeCMBLikelihood
    from cosmomc_amd.sampler import BatchedMCMC
    n = 21
    plik = NativeCMBLikelihood("PLIK_LITE", syn.make_plik_lite(12345).write(os.path.join(tmpdir, "c4p")))
    plik.nuisance_indices = [1]
    rng = np.random.default_rng(2121)                 # synthetic nuisance posterior (same on every rank)
    width = np.concatenate([[0.0025], rng.uniform(0.05, 2.0, n - 1)])
    A = rng.standard_normal((n - 1, n - 1))
    corr = A @ A.T / (n - 1) + np.eye(n - 1)
    d = np.sqrt(np.diag(corr))
    corr = corr / d[:, None] / d[None, :]
    cov = np.zeros((n, n))
    cov[0, 0] = 1.0                                   # calPlanck: left to plik_lite and its prior
    cov[1:, 1:] = corr * np.outer(width[1:], width[1:])
    P0 = np.concatenate([[1.0], rng.uniform(-1.0, 1.0, n - 1)])
    pmin, pmax = P0 - 20 * width, P0 + 20 * width
    pmin[0], pmax[0] = 0.9, 1.1
    pm, ps = np.zeros(n), np.zeros(n)
    pm[0], ps[0] = 1.0, 0.0025
    used = list(range(1, n + 1))
    smp = BatchedMCMC(W, n, used, [used], 0, pmin, pmax, pm, ps, propose_scale=2.4, seed_ij=4004 + rank,
                      seed_kl=9373, first_walker=rank * W)
    smp.set_covariance(np.diag(width ** 2))
    smp.set_test_gaussian(cov, P0)
    th = torch.tensor(syn.walker_theory(1, n_fields=3, ld_field=2512), device="cuda")
    smp.add_likelihood(plik, th.expand(W, th.shape[1], th.shape[2]))
    g = syn.gaussians(123 + rank, W * n).reshape(W, n)
    smp.set_start(np.clip(P0 + 2 * width * g, pmin + 1e-9, pmax - 1e-9))
    smp.step(5, fast_only=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    smp.step(steps, fast_only=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    out = {"workload": "plik_lite_TTTEEE + correlated 20-d Gaussian nuisance posterior (full plik's 21 fast "
                       "parameters as a sampler-throughput stand-in: clik absent), one 21-parameter fast block, "
                       "one shared slow point",
           "walkers_total": W * world, "evals_per_s": W * world * steps / dt, "ms_per_step": dt / steps * 1e3}
    out["avg_kernel_us"], out["kernel_us_per_step"] = kernel_profile(smp, 42, per_step=True)
    if seconds > 0:
        out.update(run_to_convergence(smp, 0, n, seconds, world, 60 * 40 * n))
    return out


BK15_DATASET = "BK15/BK15_dust.dataset"
BK15_MAPS = "BK15_95_B BK15_150_B BK15_220_B W023_B P030_B W033_B P044_B P070_B P100_B P143_B P217_B P353_B"


def config5_run(W, rank, world, tmpdir, seconds, steps=100):
    """BASELINE configs[4]: BK15 (12 B maps x 9 bins, HL, batch3/BK15.ini selection;
    the reference does not ship its covariance, a synthetic one of the file's
    shape is used) + plik_lite TTTEEE jointly, on one shared cached slow point.
    Fast parameters: calPlanck and the seven BK15.ini foreground parameters
    (BBdust, BBsync, BBalphadust, BBbetadust, BBalphasync, BBbetasync,
    BBdustsynccorr, with its ranges and Gaussian priors); the rest of the 16 BK
    nuisances fixed as in BK15.ini.  Reports fast-step throughput and R-1 vs
    wall-clock with the cross-GPU exchange every 40 x n_used samples."""
    import torch
    from cosmomc_amd import synthetic as syn
    from cosmomc_amd.likelihood import NativeCMBLikelihood
    from cosmomc_amd.sampler import BatchedMCMC
    rd = extract_refdata(os.path.join(tmpdir, "c5"))
    syn.write_bk15_covmat(os.path.join(rd, "BK15"))
    plik = NativeCMBLikelihood("PLIK_LITE", syn.make_plik_lite(12345).write(os.path.join(tmpdir, "c5p")))
    bk = NativeCMBLikelihood("BKPLANCK", os.path.join(rd, BK15_DATASET), {"maps_use": BK15_MAPS})
    plik.nuisance_indices = [1]
    bk.nuisance_indices = list(range(2, 18))
    #        calPlanck BBdust BBsync adust bdust  Tdust async  bsync  corr  EEd  EEs  Dd   Ds   gc   g95  g150 g220
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
    # blocks as the reference's SetFastSlowParams makes them for this list
    # (block_fast_likelihood_params, BaseParameters.f90:360-418): no theory
    # parameter varies (one cached slow point), plik_lite then BK15
    from cosmomc_amd.likelihood import LikelihoodList
    from cosmomc_amd.params import set_fast_slow_params
    ll = LikelihoodList()
    ll.add(plik)
    ll.add(bk)
    ll.add_nuisance_parameters([])
    varying = [i + 1 in used for i in range(17)]
    blk = set_fast_slow_params(17, varying, list(ll), num_theory_params=0)
    # starting proposal: a diagonal guess of the posterior widths (no covmat; the
    # reference then learns the proposal freely, covariance_is_diagonal)
    width = np.array([0.0025, 0.5, 1.0, 0.1, 0.1, 0.1, 0.3, 0.2])
    smp = BatchedMCMC(W, 17, used, blk.param_blocks, blk.slow_block_max, pmin, pmax, pm, ps, propose_scale=2.4,
                      seed_ij=3003 + rank, seed_kl=9373, first_walker=rank * W)
    smp.set_covariance(np.diag(width ** 2))
    th = torch.tensor(syn.walker_theory(1, n_fields=10, ld_field=2512), device="cuda")
    th = th.expand(W, th.shape[1], th.shape[2])       # one cached slow point for everyone
    smp.add_likelihood(plik, th)
    smp.add_likelihood(bk, th)
    start = np.tile(P0, (W, 1))
    g = syn.gaussians(91 + rank, W * 8).reshape(W, 8)
    for c, i in enumerate([u - 1 for u in used]):
        start[:, i] = np.clip(P0[i] + 2 * width[c] * g[:, c], pmin[i] + 1e-9, pmax[i] - 1e-9)
    smp.set_start(start)
    smp.step(5, fast_only=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    smp.step(steps, fast_only=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    out = {"workload": "BK15 (12 B maps x 9 bins, HL, synthetic covariance) + plik_lite_TTTEEE joint, "
                       "8 fast parameters (calPlanck + 7 BK15 foreground), one shared slow point",
           "param_blocks": blk.param_blocks,
           "walkers_total": W * world, "evals_per_s": W * world * steps / dt, "ms_per_step": dt / steps * 1e3,
           "avg_kernel_us": kernel_profile(smp, 20)}
    if seconds > 0:
        out.update(run_to_convergence(smp, 0, len(used), seconds, world, 100 * 40 * len(used)))
    return out


def host_cores():
    """Cores this job may use: the affinity mask, capped by the cgroup CPU
    quota (cpu.max) when one is set -- on the GPU box nproc shows the whole
    machine while the job's share is a quota."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return (min(n, quota) if quota else n), n, quota


def node_physical_cores():
    """Physical cores of the whole node (unique (physical id, core id) pairs in
    /proc/cpuinfo), whatever share of them this job may use."""
    pairs, phys, core = set(), None, None
    try:
        for line in open("/proc/cpuinfo"):
            k, _, v = line.partition(":")
            k = k.strip()
            if k == "physical id":
                phys = v.strip()
            elif k == "core id":
                core = v.strip()
            elif not k and phys is not None:
                pairs.add((phys, core))
                phys = core = None
        if phys is not None:
            pairs.add((phys, core))
    except OSError:
        return None
    return len(pairs) or None


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(seconds, lensing=True, repeats=5):
    """The reference's own plik_lite (+ lensing) LogLike (oracle/_ref/plik_bench,
    compiled from /root/reference with the reference's -O3 -ffast-math flags)
    on this host's cores: one single-threaded process per core (CosmoMC's
    one chain per MPI rank, OPENBLAS_NUM_THREADS=1), `repeats` timed rounds of
    `seconds` each, median of the per-round totals.  Falls back to
    the C restatement (oracle/liboracle.so, kind "port") when _ref is absent."""
    from cosmomc_amd import synthetic as syn
    P, n_aff, quota = host_cores()
    exe = os.path.join(ROOT, "oracle", "_ref", "plik_bench")
    data = syn.make_plik_lite(12345)
    Wc = 16
    th = syn.walker_theory(Wc, n_fields=3)
    cal = syn.walker_calibrations(Wc)
    host = {"cpu_model": cpu_model(), "affinity_cores": n_aff, "cgroup_quota_cores": quota,
            "node_physical_cores": node_physical_cores(), "node_logical_cpus": os.cpu_count()}
    with tempfile.TemporaryDirectory() as td:
        ds = data.write(td)
        if os.path.exists(exe):
            ini = os.path.join(td, "l.ini")
            with open(ini, "w") as f:
                f.write(f"cmb_dataset[PLIK_LITE] = {ds}\n")
                if lensing:
                    f.write(f"cmb_dataset[lensing] = {os.path.join(extract_refdata(td), LENS_DATASET)}\n")
            th = syn.walker_theory(Wc, n_fields=10 if lensing else 3)
            th.tofile(os.path.join(td, "t.bin"))
            cal.tofile(os.path.join(td, "n.bin"))
            env = dict(os.environ, OPENBLAS_NUM_THREADS="1", OMP_NUM_THREADS="1")
            cmd = [exe, ini, os.path.join(td, "t.bin"), os.path.join(td, "n.bin"), str(Wc), "2508",
                   str(th.shape[1]), "1", str(seconds)]
            totals = []
            for _ in range(repeats):
                procs = [subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env) for _ in range(P)]
                rates = []
                for pr in procs:
                    out, _ = pr.communicate(timeout=120)
                    n, t, _s = out.split()
                    rates.append(float(n) / float(t))
                totals.append(float(sum(rates)))
            what = "TPlikLiteLikelihood_LogLike + CMBLikes_LogLike (lensing)" if lensing else \
                "TPlikLiteLikelihood_LogLike"
            med = float(np.median(totals))
            pc = node_physical_cores()
            return {"value": med, "unit": "evals/s", "cores": P, "kind": "reference",
                    "per_core_evals_per_s": med / P,
                    "node_estimate_evals_per_s": (med / P * pc) if pc else None,
                    "node_estimate_note": "per-core rate x the node's physical cores (linear; not measured: "
                                          "the job may use only `cores` of them)",
                    "repeats": [round(x, 1) for x in totals], "host": host,
                    "flags": "amdflang -O3 -ffast-math -march=x86-64-v3 (reference source/Makefile:60 "
                             "-O3 -ffast-math -march=native) + OpenBLAS 1 thread",
                    "sample": f"reference {what}, {P} concurrent single-thread processes (one per core of "
                              f"this job) x {seconds:g} s over {Wc} synthetic walkers, median of {repeats} rounds"}
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle as po
        orc = po.PlikLite(data)
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            orc.loglike(th[n % Wc], cal[n % Wc])
            n += 1
        dt = time.perf_counter() - t0
        return {"value": n / dt, "unit": "evals/s", "cores": 1, "kind": "port", "host": host,
                "sample": f"C restatement oracle/liboracle.so (plik_lite only), 1 thread, {seconds:g} s"}


PLIK_RANGES = {"TT": (30, 2508), "TE": (30, 1996), "EE": (30, 1996)}   # plik_lite's binned l (CMB.f90:315-325)


def lensing_window_bytes(refdir, with_plik=False):
    """Algorithmic bytes of one lensing window-contraction launch, split into
    per-walker theory bytes (each field's D_l over the union of its windows'
    nonzero l ranges, read once) and per-launch window bytes (nonzero weights,
    read once): CMBlikes.f90:1230-1256 over the consext8 windows.  with_plik:
    the fused window pass (theorypass.hip), which also reads plik_lite's binned
    l (the union per field, once) and its 6413 weights."""
    base = os.path.join(refdir, LENS_DATASET.replace(".dataset", ""))
    ranges = {}
    wbytes = 0
    for sub, fields in (("_window", ["PP"]), ("_lens_delta_window", ["TT", "EE", "TE", "PP"])):
        for b in range(1, 10):
            a = np.loadtxt(f"{base}{sub}/window{b}.dat", ndmin=2)
            for k, f in enumerate(fields):
                nz = np.nonzero(a[:, 1 + k])[0]
                if len(nz):
                    lo, hi = int(a[nz[0], 0]), int(a[nz[-1], 0])
                    r = ranges.get(f, (lo, hi))
                    ranges[f] = (min(r[0], lo), max(r[1], hi))
                    wbytes += 8 * len(nz)
    if with_plik:
        for f, (lo, hi) in PLIK_RANGES.items():
            r = ranges.get(f, (lo, hi))
            ranges[f] = (min(r[0], lo), max(r[1], hi))     # the lensing ranges contain or adjoin plik's
        wbytes += 8 * N_L
    per_walker = 8 * sum(hi - lo + 1 for lo, hi in ranges.values())
    return per_walker, wbytes


def pmc_traffic(kernel, W):
    """HBM bytes per launch of ``kernel`` from the committed rocprofv3 PMC pass
    (tools/gpu_pmc.sh -> tools/pmc_summary.py, FETCH_SIZE x2 + WRITE_SIZE per the
    MI355X guide) when it was taken at this walker count; else null."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None
    if d.get("walkers") != W:
        return None, None
    symbols = {"plik_quadform_ksplit": ("quadform_ksplit<false>", "quadform_ksplit"),   # profiler label -> kernel
               "cmbl_window_kernel": ("cmbl_window_direct",),
               "theory_window_kernel": ("theory_window_vec<2, 0>", "theory_window_kernel<2>", "theory_window_kernel<4>",
                                        "theory_window_kernel"),
               "mh_step_kernel": ("mh_step_kernel<true, true>", "mh_step_kernel")}.get(kernel, (kernel,))
    t = next((d["per_launch"][k] for k in symbols if k in d["per_launch"]), None)
    if not t:
        return None, None
    return t["fetch_bytes"] + t["write_bytes"], "profiles/pmc_traffic.json"


def kernel_roofline(kern, avg_ms, W, fused_bytes, lens_bytes):
    """Roofline of one library kernel on this workload: its algorithmic work
    per launch (bytes for HBM-bound kernels, flops for MFMA-bound ones, both
    for the unified step launch, which runs an HBM-bound pass and an
    MFMA-bound quadratic form side by side) over its average launch time (HIP
    events).  Every library kernel has an entry, so frac is never null."""
    t = avg_ms * 1e-3
    pass_bytes = W * fused_bytes[0] + fused_bytes[1]          # theory rows (each read once) + window weights
    qf_flops = W * FLOPS_QUADFORM                               # 2 N_b^2 + 2 N_b per walker (the kernel does ~half)
    hbm = {   # bytes per launch
        "plik_bin_delta": W * BYTES_BIN + 8 * N_B * W,
        "cmbl_window_kernel": W * lens_bytes[0] + lens_bytes[1],
        "theory_window_kernel": pass_bytes + 8 * N_B * W,      # + plik's Delta rows written
        "mh_kernel": W * 1024,                                 # ~1 KB of walker state read + written (latency-bound)
        # the unified step launch, algorithmic bytes only: every walker's theory rows read once, the
        # window weights and C^-1 once (not the raw sums the pass hands to the next launch's
        # quadratic form, nor the ~1 KB per walker of Metropolis state)
        "mh_step_kernel": pass_bytes + 8 * N_B * N_B,
    }
    mfma = {"plik_quadform_ksplit": qf_flops, "plik_quadform_corun": qf_flops, "mh_step_kernel": qf_flops,
            "mh_step_last": qf_flops}
    parts = {}
    if kern in hbm:
        a = hbm[kern] / t / 1e9
        parts["hbm"] = {"achieved": a, "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": a / PEAK_HBM_GBS,
                        "bytes_per_launch": hbm[kern]}
    if kern in mfma:
        a = mfma[kern] / t / 1e12
        parts["mfma"] = {"achieved": a, "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s", "frac": a / PEAK_FP64_TFLOPS,
                         "flops_per_launch": mfma[kern]}
    if not parts:        # a kernel of another leg (CMBlikes HL, BK): priced as HBM on its launch time only
        parts["hbm"] = {"achieved": None, "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": None}
    bound = max(parts, key=lambda k: parts[k]["frac"] or 0.0)
    p = parts[bound]
    roof = {"kernel": kern, "bound": bound, "achieved": p["achieved"], "peak": p["peak"], "unit": p["unit"],
            "frac": p["frac"], "traffic": None, "avg_launch_us": avg_ms * 1e3}
    if len(parts) > 1:
        roof["components"] = parts
        # the launch's time against its two components run back to back at their
        # peaks (frac above is the larger one alone, i.e. against perfect overlap)
        roof["components_serial_frac"] = sum(q["frac"] for q in parts.values())
    return roof


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args):
    """`bench.py --gpus N` (N > 1) started as a plain process: start the N
    ranks as child processes (torch.distributed.run, one per GPU, rendezvous on
    127.0.0.1) and return their exit code.  Runs before anything touches the
    GPU; device_count() does not initialise it on this image.  With the nccl
    (RCCL) backend every rank needs its own device, so N above the device count
    is refused; gloo rehearses N ranks on fewer devices."""
    import torch
    ndev = torch.cuda.device_count()
    if args.dist_backend == "nccl" and args.gpus > ndev:
        sys.exit(f"bench.py: --gpus {args.gpus} needs {args.gpus} GPUs for the nccl (RCCL) backend, "
                 f"this node has {ndev}; use --dist-backend gloo to rehearse ranks on fewer devices")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.run(cmd, env=env).returncode


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    if "WORLD_SIZE" in os.environ and args.gpus not in (1, world):
        sys.exit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    import torch
    import torch.distributed as dist
    from cosmomc_amd import _native as N

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    N.require_gpu()
    ndev = torch.cuda.device_count()
    if args.dist_backend == "nccl" and world > 1 and local >= ndev:
        raise SystemExit(f"rank {rank}: LOCAL_RANK {local} has no GPU of its own ({ndev} visible) for RCCL")
    dev = local % max(1, ndev)                         # gloo rehearsals may put several ranks on one GPU
    torch.cuda.set_device(dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(args.dist_backend)
    W = args.walkers
    devices = [dev]
    if world > 1:                                      # which device each rank ran on (reported)
        t = torch.tensor([dev], dtype=torch.int64, device="cuda" if args.dist_backend == "nccl" else "cpu")
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(parts, t)
        devices = [int(p.item()) for p in parts]
    with tempfile.TemporaryDirectory() as td:
        smp, likes, theory, _ = build_problem(W, rank, td, args.groups, lensing=not args.no_lensing)
        lens_bytes = lensing_window_bytes(os.path.join(td, "refdata")) if not args.no_lensing else (0, 0)
        fused_bytes = lensing_window_bytes(os.path.join(td, "refdata"), True) if not args.no_lensing else (0, 0)

        def barrier():
            if world > 1:
                dist.barrier()

        smp.step(args.warmup, fast_only=True)
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        smp.step(args.steps, fast_only=True)
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([dt], dtype=torch.float64, device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        evals = world * W * args.steps

        # roofline pass: same steps with per-kernel HIP events on the launch stream
        N.profile_reset()
        N.profile_enable(True)
        smp.step(args.steps, fast_only=True)
        torch.cuda.synchronize()
        N.profile_enable(False)
        kern = {k: N.profile_read(k) for k in KERNELS}
        kern = {k: v for k, v in kern.items() if v[1]}
        _, _, _, nacc = smp.state()
        acc_rate = float(nacc.sum()) / (W * (args.warmup + 2 * args.steps))
        cache = None
        if args.cache_steps > 0 and not args.no_lensing:
            cache = binned_cache_run(smp, W, world, args.cache_steps)
        conv = None
        if args.converge_seconds > 0:
            conv = convergence_run(W, rank, world, td, args.converge_seconds, lensing=not args.no_lensing)
        c1 = None
        if args.config1_seconds >= 0:
            c1 = config1_run(256, rank, world, td, args.config1_seconds)
        c4 = None
        if args.config4_seconds >= 0:
            c4 = config4_run(512, rank, world, td, args.config4_seconds)
        c5 = None
        if args.config5_seconds >= 0:
            c5 = config5_run(W, rank, world, td, args.config5_seconds)
        c2d = None
        if args.drag_seconds >= 0 and not args.no_lensing:
            c2d = drag_run(W, rank, world, td, args.drag_seconds)

    dom = max(kern, key=lambda k: kern[k][0])
    avg_ms = {k: (v[0] / v[1] if v[1] else None) for k, v in kern.items()}
    roof = kernel_roofline(dom, avg_ms[dom], W, fused_bytes, lens_bytes)
    # the step as a whole against SURVEY 8(d)'s ceiling: evals/s x F / min(P_FP64, AI x BW)
    per_gpu = evals / dt / world
    ai = FLOPS_EVAL / (BYTES_BIN + 8 * (N_B * N_B + 2479 + N_B) / W)
    ceil_flops = min(PEAK_FP64_TFLOPS * 1e12, ai * PEAK_HBM_GBS * 1e9)
    roof["step"] = {"achieved_tflops": per_gpu * FLOPS_EVAL / 1e12, "ceiling_tflops": ceil_flops / 1e12,
                    "frac": per_gpu * FLOPS_EVAL / ceil_flops,
                    "note": "per GPU, SURVEY 8(d): F = 766,816 flop/eval, B = 51,320 + 3,030,888 / W bytes/eval "
                            "(plik_lite only; the lensing likelihood's work is not counted)"}
    roof["avg_kernel_us"] = {k: (v * 1e3 if v else None) for k, v in avg_ms.items()}
    roof["traffic"], roof["traffic_source"] = pmc_traffic(dom, W)

    if rank == 0:
        out = {
            "metric": METRIC, "value": evals / dt, "unit": "evals/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": ("plik_lite_TTTEEE + Planck2018 lensing" if not args.no_lensing else
                                    "plik_lite_TTTEEE") +
                                   " fast-parameter Metropolis step (BASELINE configs[2]" +
                                   (" minus lowl" if not args.no_lensing else " minus lowl/lensing") +
                                   "): GetProposalFast + native plik_lite (613 bins, l<=2508, full binning + "
                                   "quadratic form)" + (" + CMBlikes lensing (9 bins, linear correction)"
                                                        if not args.no_lensing else "") +
                                   " + calPlanck prior + accept",
                       "walkers_per_gpu": W, "stream_groups": args.groups, "global_walkers": W * world, "nbins": N_B, "lmax": 2508,
                       "parallelism": f"walkers sharded over {world} rank(s), no per-step collective",
                       "rank_devices": devices, "dist_backend": args.dist_backend if world > 1 else None,
                       "accept_rate": acc_rate},
            "roofline": roof,
        }
        if conv is not None:
            out["convergence"] = conv
        if cache is not None:
            out["binned_cache"] = cache
        if c1 is not None:
            out["config1_tt"] = c1
        if c4 is not None:
            out["config4_fast21"] = c4
        if c5 is not None:
            out["config5_bk15_plik"] = c5
        if c2d is not None:
            out["config2_drag"] = c2d
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.cpu_seconds, lensing=not args.no_lensing)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
