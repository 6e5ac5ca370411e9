"""ORACLE TEST INFRASTRUCTURE -- generates tests/golden/*.json from the compiled
reference (oracle/_ref, built by `make -C oracle ref` from /root/reference).

Runs only in the development container: it needs /root/reference to build
oracle/_ref.  The built oracle/_ref binaries do travel to the GPU box (they are
git-ignored, not gpurun-ignored), where bench.py's cpu_baseline leg times
plik_bench; nothing on the box regenerates fixtures.  Each fixture records the
seeds that regenerate its inputs through cosmomc_amd.synthetic, plus the
reference outputs; the committed fixtures are small, the inputs are rebuilt on
both sides.

    python oracle/gen_golden.py            # all fixtures
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
from cosmomc_amd import synthetic as syn  # noqa: E402

REF_DIR = os.path.join(HERE, "_ref")
GOLDEN = os.path.join(ROOT, "tests", "golden")


def run_cmb_harness(ini_text: str, theory: np.ndarray, nuis: np.ndarray, workdir: str,
                    derived: bool = False) -> np.ndarray:
    """theory [W, nfield, lmax+1]; nuis [W, n_nuis] -> reference -lnL [W]
    (derived: the harness also writes derivedParameters to workdir/derived.txt)."""
    W, nfield, nl = theory.shape
    ini = os.path.join(workdir, "likes.ini")
    with open(ini, "w") as f:
        f.write(ini_text)
    th = os.path.join(workdir, "theory.bin")
    nu = os.path.join(workdir, "nuis.bin")
    out = os.path.join(workdir, "out.txt")
    np.ascontiguousarray(theory, dtype="<f8").tofile(th)
    np.ascontiguousarray(nuis, dtype="<f8").tofile(nu)
    cmd = [os.path.join(REF_DIR, "plik_harness"), ini, th, nu, str(W), str(nl - 1), str(nfield),
           str(nuis.shape[1]), out] + ([os.path.join(workdir, "derived.txt")] if derived else [])
    env = dict(os.environ, OPENBLAS_NUM_THREADS="1", OMP_NUM_THREADS="1")
    if os.path.exists(out):
        os.remove(out)                # a Fortran STOP exits 0: never read a stale result
    subprocess.run(cmd, check=True, cwd=workdir, env=env, stdout=subprocess.DEVNULL)
    res = np.loadtxt(out, ndmin=1)
    if res.size != W:
        raise RuntimeError(f"reference harness wrote {res.size} of {W} results")
    return res


PLIK_CASES = [
    # name, override lines (cmb_dataset[PLIK_LITE,key] = value), walkers
    ("plik_lite_TTTEEE", {}, 8),
    ("plik_lite_TT", {"use_cl": "TT"}, 8),
    ("plik_lite_TE", {"use_cl": "TE"}, 4),
    ("plik_lite_TTEE", {"use_cl": "TT EE"}, 4),
    ("plik_lite_TTTEEE_Lrange", {"bins_for_L_range": "100 1500"}, 4),
]


def gen_plik(data_seed=12345, theory_seed=0xC05A0C, cal_seed=0xCA1):
    data = syn.make_plik_lite(data_seed)
    out = {"generator": "cosmomc_amd.synthetic", "data_seed": data_seed,
           "theory_seed": theory_seed, "cal_seed": cal_seed, "cases": {}}
    with tempfile.TemporaryDirectory() as td:
        ds = data.write(td)
        for name, over, W in PLIK_CASES:
            lines = [f"cmb_dataset[PLIK_LITE] = {ds}"]
            lines += [f"cmb_dataset[PLIK_LITE,{k}] = {v}" for k, v in over.items()]
            theory = syn.walker_theory(W, seed=theory_seed, n_fields=3)
            cal = syn.walker_calibrations(W, seed=cal_seed)
            cal[0] = 1.0            # the survey's cal = 1 anchor
            lnl = run_cmb_harness("\n".join(lines) + "\n", theory, cal[:, None], td)
            out["cases"][name] = {"overrides": over, "walkers": W, "cal": cal.tolist(),
                                  "minus_lnL": lnl.tolist()}
            print(f"{name:28s} W={W}  -lnL[0..2] = {lnl[:3]}")
    with open(os.path.join(GOLDEN, "plik_lite_ref.json"), "w") as f:
        json.dump(out, f, indent=1)


def run_rng(mode: str, cfg_text: str, workdir: str) -> list[str]:
    cfg = os.path.join(workdir, "cfg.txt")
    out = os.path.join(workdir, "rng_out.txt")
    with open(cfg, "w") as f:
        f.write(cfg_text)
    subprocess.run([os.path.join(REF_DIR, "rng_harness"), mode, cfg, out], check=True, cwd=workdir,
                   stdout=subprocess.DEVNULL)
    with open(out) as f:
        return f.read().split("\n")


def _fmt(a):
    return " ".join(f"{x:.17e}" for x in np.ravel(a))


# chain configurations: (name, n_used, blocks, slow_block_max, oversample_fast, propose_scale, fast_only, steps,
#                        extra) with extra = {"fixed": k fixed parameters appended after the used ones,
#                        "include_fixed": include_fixed_parameter_priors, "lincomb": number of
#                        linear-combination priors (BaseParameters.f90:184-201), "burn_in": the
#                        sampler's burn_in (MCMC.f90:39, default 2)}.  fast_only: 0 ->
#                        TMetropolisSampler_GetNewSample, 1 -> FastParameterSample, 2 -> fast dragging.
CHAIN_CASES = [
    # config 1: 6-D Gaussian, test_likelihood, one (slow) block, no fast/slow split
    ("gauss6_single_block", 6, [[1, 2, 3, 4, 5, 6]], 1, 1, 2.4, 0, 400, {}),
    # slow 2 + fast 3 + fast 1, oversample_fast 2, full GetProposal cycle
    ("gauss6_blocked", 6, [[1, 2], [3, 4, 5], [6]], 1, 2, 2.4, 0, 400, {}),
    # fast-only steps (FastParameterSample path) with propose_scale 1.9 (batch3/common.ini)
    ("gauss6_fast_only", 6, [[1, 2], [3, 4, 5], [6]], 1, 1, 1.9, 1, 400, {"burn_in": 0}),
    # 1-D block of calPlanck-like width (sign flip RotMatrix branch, n=1)
    ("gauss3_n1_blocks", 3, [[1], [2], [3]], 1, 3, 2.4, 0, 300, {"burn_in": 5}),
    # fast dragging (TFastDraggingSampler, fast_only = 2): slow 2 + fast 3 + fast 1, drag every 2nd step
    ("gauss6_drag", 6, [[1, 2], [3, 4, 5], [6]], 1, 2, 2.4, 2, 240, {}),
    # dragging every step (oversample_fast 1), one fast parameter (interp_steps 4)
    ("gauss4_drag_every_step", 4, [[1, 2, 3], [4]], 1, 1, 2.0, 2, 200, {"burn_in": 1}),
    # BASELINE configs[3] shape: 6 slow + one 21-parameter fast block (full plik's foreground
    # nuisance set), fast-only steps; rotations of 21x21 regenerated every 21 draws
    ("gauss27_fast21_fast_only", 27, [list(range(1, 7)), list(range(7, 28))], 1, 1, 1.9, 1, 320,
     {"lincomb": 1, "fixed": 1}),
    # same parameters, full GetProposal cycle with oversample_fast 3
    ("gauss27_fast21_os3", 27, [list(range(1, 7)), list(range(7, 28))], 1, 3, 2.4, 0, 320,
     {"lincomb": 1, "burn_in": 5}),
    # the 21 fast parameters split 12 + 9 (block_fast_likelihood_params: two likelihoods),
    # a linear-combination prior (batch2/plik_dx11dr2_HM_v18_TT.ini:16-17 SZComb) and fixed
    # parameters whose priors count (include_fixed_parameter_priors = T)
    ("gauss27_fast12_9_lincomb", 27, [list(range(1, 7)), list(range(7, 19)), list(range(19, 28))], 1, 3, 2.4, 0,
     320, {"lincomb": 2, "fixed": 2, "include_fixed": 1}),
    # 40 used parameters: slow 6 + semi-slow 4 + fast 21 + fast 9, oversample_fast 3,
    # fixed-parameter priors present but not counted (include_fixed_parameter_priors = F)
    ("gauss40_slow_fast", 40, [list(range(1, 7)), list(range(7, 11)), list(range(11, 32)), list(range(32, 41))],
     2, 3, 2.4, 0, 300, {"lincomb": 1, "fixed": 2}),
    # dragging with a 21-parameter fast block (interp_steps = 64)
    ("gauss27_fast21_drag", 27, [list(range(1, 7)), list(range(7, 28))], 1, 2, 2.4, 2, 40, {"lincomb": 1}),
]


def chain_problem(n: int, seed: int, extra=None):
    """The case's test Gaussian (cosmomc_amd.synthetic.chain_problem: the tests
    rebuild it from the seed, so the fixture stores only results)."""
    return syn.chain_problem(n, seed, extra)


def problem_sums(prob) -> list[float]:
    """Checksums of a chain problem, stored with the fixture so a host that
    rebuilds it can confirm it is the problem the reference ran on."""
    cov, center, pmin, pmax, pmean, pstd, P0, lin = prob
    return [float(np.sum(cov)), float(np.sum(np.abs(cov))), float(np.sum(center)), float(np.sum(pmin)),
            float(np.sum(pmax)), float(np.sum(pmean)), float(np.sum(pstd)), float(np.sum(P0))] + \
        [float(lc["mean"]) for lc in lin] + [float(lc["std"]) for lc in lin]


def stored_steps(steps: int, n: int) -> list[int]:
    """Steps (0-based) whose trial/current -lnL and point the fixture keeps:
    the first three, every `every`-th and the last (the fixture stays under
    100 KB; the accept decision of every step is kept)."""
    every = max(1, steps // (16 if n <= 8 else 8))
    return sorted({0, 1, 2, steps - 1} | {k for k in range(steps) if (k + 1) % every == 0})


def gen_rng():
    import hashlib
    out = {"kat": None, "streams": {}, "chains": {}}
    with tempfile.TemporaryDirectory() as td:
        out["kat"] = [float(x) for x in run_rng("kat", "", td) if x.strip()]
        for ij, kl in ((1802, 9373), (1234, 5678), (31328, 30081)):
            n, nidx, nrot = 60, 12, 5
            lines = [x for x in run_rng("stream", f"{ij} {kl} {n} {nidx} {nrot}\n", td) if x.strip()]
            vals = [float(x) for x in lines]
            out["streams"][f"{ij}_{kl}"] = {
                "ij": ij, "kl": kl, "ranmar": vals[:n], "gaussian1": vals[n:2 * n],
                "randexp1": vals[2 * n:3 * n], "rand_indices": [int(v) for v in vals[3 * n:3 * n + nidx]],
                "rotation": vals[3 * n + nidx:], "nidx": nidx, "nrot": nrot}
        for ci, (name, n, blocks, sbm, ovs, scale, fast_only, steps, extra) in enumerate(CHAIN_CASES):
            prob = chain_problem(n, 777 + ci, extra)
            cov, center, pmin, pmax, pmean, pstd, P0, lin = prob
            npar = len(center)
            ij, kl = 4321 + ci, 9373
            T = 1.0
            incl = int(extra.get("include_fixed", 0))
            burn = int(extra.get("burn_in", 2))
            used = list(range(1, n + 1))
            cfg = [f"{ij} {kl} {npar} {n} {steps} {fast_only} {incl} {len(lin)}",
                   f"{len(blocks)} {sbm} {ovs} {scale!r} {T!r} {burn}",
                   " ".join(str(u) for u in used),
                   " ".join(str(len(b)) for b in blocks)]
            cfg += [" ".join(str(x) for x in b) for b in blocks]
            cfg += [_fmt(cov), _fmt(center), _fmt(pmin), _fmt(pmax), _fmt(pmean), _fmt(pstd), _fmt(P0)]
            for lc in lin:
                cfg += [_fmt(lc["weights"]), f"{lc['mean']!r} {lc['std']!r}"]
            lines = [x for x in run_rng("chain", "\n".join(cfg) + "\n", td) if x.strip()]
            like0 = float(lines[0])
            rows = np.array([[float(v) for v in l.split()] for l in lines[1:]])
            assert rows.shape[0] == steps
            base = os.path.join(td, "rng_out.txt")
            with open(base + ".txt", "rb") as f:
                chain_txt = f.read()
            pts = np.loadtxt(base + ".points", ndmin=2)
            mx = open(base + ".max").read().split()
            keep = stored_steps(steps, n)
            out["chains"][name] = {
                "ij": ij, "kl": kl, "n": n, "num_params": npar, "params_used": used, "blocks": blocks,
                "slow_block_max": sbm, "oversample_fast": ovs, "propose_scale": scale, "fast_only": fast_only,
                "temperature": T, "steps": steps, "problem_seed": 777 + ci, "extra": extra,
                "include_fixed_parameter_priors": incl, "burn_in": burn, "problem_sums": problem_sums(prob),
                "like0": like0, "accept": "".join(str(int(a)) for a in rows[:, 0]),
                "stored_steps": keep, "trial_like": rows[keep, 1].tolist(), "cur_like": rows[keep, 2].tolist(),
                "P": rows[keep, 3:].tolist(),
                # the reference's own chain file (TMpiChainCollector_AddNewWeightedPoint -> IO_OutputChainRow,
                # RealFormat E16.7 settings.f90:109) and its AddNewWeightedPoint calls (mult, thin_fac)
                "chain_file": {"rows": chain_txt.count(b"\n"), "sha256": hashlib.sha256(chain_txt).hexdigest(),
                               "first_row": chain_txt.decode().splitlines()[0]},
                "weighted_points": {"count": int(pts.shape[0]) if pts.size else 0,
                                    "mult": pts[:, 0].astype(int).tolist() if pts.size else [],
                                    "thin_fac": int(pts[0, 1]) if pts.size else None},
                "num_accept": int(mx[0]), "max_like": float(mx[1])}
            nrows = chain_txt.count(b"\n")
            print(f"chain {name:26s} accept rate {rows[:, 0].mean():.3f}  final -lnL {rows[-1, 2]:.6f}  "
                  f"chain rows {nrows}")
    with open(os.path.join(GOLDEN, "rng_sampler_ref.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))


# convergence cases: (name, chains, samples per chain, n_used, centre spread, seed)
GR_CASES = [("gr_n3_m8", 8, 400, 3, 0.3, 501), ("gr_n6_m16", 16, 301, 6, 0.05, 502),
            ("gr_n2_m4", 4, 1000, 2, 1.0, 503), ("gr_n7_m32", 32, 120, 7, 0.01, 504)]


def gen_gr():
    """GelmanRubinEvalues of the compiled reference on the pooled statistics of
    synthetic chain ensembles (cosmomc_amd.synthetic.chain_ensemble)."""
    sys.path.insert(0, HERE)
    import pyoracle as po
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for name, M, T, n, spread, seed in GR_CASES:
            x = syn.chain_ensemble(M, T, n, seed, spread)
            st = po.pool_chain_statistics(list(x))
            # Fortran reads column-major: transpose so cov(i,j) is row i col j
            lines = [x_ for x_ in run_rng("gr", f"{n}\n{_fmt(st['cov'].T)}\n{_fmt(st['meanscov'].T)}\n", td)
                     if x_.strip()]
            ok = int(lines[0])
            ev = [float(v) for v in lines[1:]]
            out[name] = {"chains": M, "samples": T, "n": n, "spread": spread, "seed": seed, "ok": ok,
                         "evals": ev, "R": max(ev), "mean": st["mean"].tolist(),
                         "propose_cov": st["propose_cov"].tolist(), "cov": st["cov"].tolist(),
                         "meanscov": st["meanscov"].tolist()}
            print(f"{name}: R-1 = {max(ev):.6e}")
    with open(os.path.join(GOLDEN, "gr_ref.json"), "w") as f:
        json.dump(out, f, indent=0)


# ConfidVal cases: (name, samples, columns, ix1, ix2, limfrac, seed)
CONFID_CASES = [("confid_gauss_window", 401, 3, 200, 401, 0.025, 611), ("confid_all_0p05", 97, 2, 1, 97, 0.05, 612),
                ("confid_ties", 120, 2, 60, 120, 0.025, 613), ("confid_small", 7, 1, 3, 7, 0.3, 614)]


def gen_confid():
    """TSampleList%ConfidVal of the compiled reference (CheckLimitsConverge's
    per-chain limits) on seeded synthetic sample columns."""
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for name, ns, nc, ix1, ix2, frac, seed in CONFID_CASES:
            v = syn.gaussians(seed, ns * nc).reshape(ns, nc)
            if "ties" in name:
                v = np.round(v * 3) / 3                  # many equal values
            cfg = f"{ns} {nc} {ix1} {ix2} {frac!r}\n{_fmt(v)}\n"
            lines = [x for x in run_rng("confid", cfg, td) if x.strip()]
            lims = [[float(a) for a in l.split()] for l in lines]
            out[name] = {"samples": ns, "columns": nc, "ix1": ix1, "ix2": ix2, "limfrac": frac, "seed": seed,
                         "ties": "ties" in name, "limits": lims}
            print(f"{name}: {lims[0]}")
    with open(os.path.join(GOLDEN, "confid_ref.json"), "w") as f:
        json.dump(out, f, indent=0)


# CMBlikes cases on the reference's own data (tests/golden/refdata.tar.xz):
# (name, tag, dataset, overrides, walkers, lmax, nuisance kind)
LENS = "planck_lensing_2018/smicadx12_Dec5_ftl_mv2_ndclpp_p_teb_consext8.dataset"
BKP = "BKPlanck/BKPlanck_detset_comb_dust.dataset"
BK15 = "BK15/BK15_dust.dataset"
BK15_MAPS = "BK15_95_B BK15_150_B BK15_220_B W023_B P030_B W033_B P044_B P070_B P100_B P143_B P217_B P353_B"
CMBL_CASES = [
    ("lensing_consext8", "lensing", LENS, {}, 6, 2500, "cal"),
    ("bkplanck_3map_bins1to5", "BKPLANCK", BKP, {"maps_use": "B2K_B P217_B P353_B", "use_min": "1", "use_max": "5"},
     5, 600, "bk_fid"),
    ("bkplanck_all_maps", "BKPLANCK", BKP, {}, 4, 600, "bk_sync"),
    ("bkplanck_decorr_lin_quad", "BKPLANCK", BKP, {"lform_dust_decorr": "lin", "lform_sync_decorr": "quad"},
     3, 600, "bk_decorr"),
    ("bkplanck_EB_4map", "BKPLANCK", BKP, {"maps_use": "B2K_E B2K_B P353_E P353_B", "use_max": "7"}, 3, 600, "bk_sync"),
    ("sptsz_aberration_calprior", "SPT", "sptsz_2500d_tt/spt_s13_margfg.dataset", {}, 5, 3300, "cal_spt"),
    # BASELINE configs[4]: BK15 B-only, 12 maps x 9 bins (batch3/BK15.ini), synthetic covariance
    ("bk15_B_12maps", "BKPLANCK", BK15, {"maps_use": BK15_MAPS, "use_min": "1", "use_max": "9"}, 3, 600, "bk_sync"),
    ("bk15_B_decorr_bandcentre", "BKPLANCK", BK15, {"maps_use": BK15_MAPS}, 3, 600, "bk15_bc"),
    # calibration_param read by the base ReadIni, then the names replaced by BK's
    # nuisance_params (CMB_BK_Planck.f90:43-46): the calibration index (1) stays and
    # points at BBdust (the reference's own behaviour), with its log prior
    ("bkplanck_calparam_prior", "BKPLANCK", BKP, {"maps_use": "B2K_B P217_B P353_B", "use_max": "5",
                                                  "calibration_param": "bk_cal.paramnames",
                                                  "log_calibration_prior": "0.5"}, 3, 600, "bk_fid"),
]
BK_FID = [3.0, 0.0, -0.42, 1.59, 19.6, -0.6, -3.3, 0.0, 2.0, 1.0, 1.0, 1.0, 0.0, 0.0, 0.0, 0.0]


def cmbl_nuisance(kind, W, seed):
    g = syn.gaussians(seed, W * 16).reshape(W, 16)
    if kind == "cal":
        return 1.0 + 0.0025 * g[:, :1]
    if kind == "cal_spt":
        return 1.0 + 0.0017 * g[:, :1]
    P = np.tile(np.array(BK_FID), (W, 1))
    P[:, 0] = 3.0 + 0.5 * g[:, 0]
    P[:, 3] = 1.59 + 0.05 * g[:, 3]
    if kind in ("bk_sync", "bk_decorr"):
        P[:, 1] = 1.0 + 0.2 * np.abs(g[:, 1])
        P[:, 2] = -0.42 + 0.05 * g[:, 2]
        P[:, 4] = 19.6 + 0.5 * g[:, 4]
        P[:, 7] = 0.2 + 0.05 * g[:, 7]
    if kind == "bk15_bc":
        P[:, 1] = 1.0 + 0.2 * np.abs(g[:, 1])
        P[:, 7] = 0.2 + 0.05 * g[:, 7]
        P[:, 10] = 0.9 + 0.02 * g[:, 10]
        P[:, 11] = 0.95 + 0.02 * g[:, 11]
        P[:, 12:16] = 0.01 * g[:, 12:16]
    if kind == "bk_decorr":
        P[:, 7] = 0.0
        P[:, 10] = 0.85 + 0.02 * g[:, 10]
        P[:, 11] = 0.9 + 0.02 * g[:, 11]
    return P


def refdata_dir(td):
    import lzma
    import tarfile
    import io
    d = os.path.join(td, "refdata")
    with open(os.path.join(GOLDEN, "refdata.tar.xz"), "rb") as f:
        tar = tarfile.open(fileobj=io.BytesIO(lzma.decompress(f.read())))
        try:
            tar.extractall(d, filter="data")
        except TypeError:
            tar.extractall(d)
    syn.write_refdata_extras(d)
    return d


def gen_cmblikes():
    out = {"theory_seed": 0xC05A0C, "cases": {}}
    with tempfile.TemporaryDirectory() as td:
        data = refdata_dir(td)
        for ci, (name, tag, ds, over, W, lmax, kind) in enumerate(CMBL_CASES):
            th = syn.walker_theory(W, seed=out["theory_seed"] + 1000 * ci, lmax=lmax)
            nu = cmbl_nuisance(kind, W, 4242 + ci)
            ini = f"cmb_dataset[{tag}] = {os.path.join(data, ds)}\n" + \
                "".join(f"cmb_dataset[{tag},{k}] = {v}\n" for k, v in over.items())
            ref = run_cmb_harness(ini, th, nu, td)
            out["cases"][name] = {"tag": tag, "dataset": ds, "overrides": over, "walkers": W, "lmax": lmax,
                                  "theory_seed": out["theory_seed"] + 1000 * ci, "nuis": nu.tolist(),
                                  "minus_lnL": ref.tolist()}
            print(f"{name:28s} -lnL[0] = {ref[0]:.10f}")
    with open(os.path.join(GOLDEN, "cmblikes_ref.json"), "w") as f:
        json.dump(out, f, indent=1)


# SMICA (TSmica_planck, CMBlikes.f90:1262-1339) on the synthetic dataset
# (cosmomc_amd.synthetic.make_smica): (name, like_approx, dataset overrides, walkers, n1run free)
SMICA_CASES = [
    ("smica_gauss", "gaussian", {}, 4, False),
    ("smica_gauss_run", "gaussian", {}, 4, True),
    ("smica_gauss_calname", "gaussian", {"calibration_paramname": "cal_smica"}, 4, True),
    ("smica_hl_aber_calname", "HL", {"calibration_paramname": "cal_smica", "aberration_coeff": "0.0012"}, 3, True),
    # calibration_param loaded by the base ReadIni, then replaced by nuisance_params: its
    # calibration index (1) stays and points at A1_smica (the reference's own behaviour)
    ("smica_calparam_override", "gaussian", {"calibration_param": "smica_cal.paramnames",
                                             "log_calibration_prior": "0.0025"}, 3, True),
    ("smica_calname_unknown", "gaussian", {"calibration_paramname": "no_such_param"}, 3, False),
]


def smica_nuisance(W, seed, run):
    g = syn.gaussians(seed, W * 6).reshape(W, 6)
    c = np.array(list(syn.SMICA_FG) + [1.0])
    sd = np.array([5.0, 0.1, 0.3 if run else 0.0, 3.0, 0.1, 0.0025])
    return c[None, :] + g * sd[None, :]


def run_cmb_harness_derived(ini_text, theory, nuis, workdir):
    """run_cmb_harness, also returning derivedParameters per walker."""
    W, nfield, nl = theory.shape
    lnl = run_cmb_harness(ini_text, theory, nuis, workdir, derived=True)
    with open(os.path.join(workdir, "derived.txt")) as f:
        der = [[float(x) for x in line.split()] for line in f][:W]
    return lnl, der


def gen_smica():
    out = {"theory_seed": 0xC05A0C, "generator": "cosmomc_amd.synthetic.make_smica", "cases": {}}
    with tempfile.TemporaryDirectory() as td:
        for ci, (name, approx, over, W, run) in enumerate(SMICA_CASES):
            path = syn.make_smica().write(os.path.join(td, name), like_approx=approx)
            th = syn.walker_theory(W, seed=out["theory_seed"] + 10 * ci, lmax=2508, n_fields=6)
            nu = smica_nuisance(W, 6060 + ci, run)
            ini = f"cmb_dataset[SMICA] = {path}\n" + "".join(f"cmb_dataset[SMICA,{k}] = {v}\n" for k, v in over.items())
            lnl, der = run_cmb_harness_derived(ini, th, nu, td)
            out["cases"][name] = {"like_approx": approx, "overrides": over, "walkers": W, "lmax": 2508,
                                  "theory_seed": out["theory_seed"] + 10 * ci, "nuis": nu.tolist(),
                                  "minus_lnL": lnl.tolist(), "derived": der}
            print(f"{name:28s} -lnL = {lnl}  derived[0] = {der[0]}")
    with open(os.path.join(GOLDEN, "smica_ref.json"), "w") as f:
        json.dump(out, f, indent=1)


# SPTpol cases on the synthetic datasets (cosmomc_amd.synthetic.make_sptpol_*):
# (name, tag, dataset overrides, walkers)
SPTPOL_CASES = [
    ("teee_default", "SPTPOL_TEEE", {}, 4),
    ("teee_aberration_priors", "SPTPOL_TEEE",
     {"correct_aberration": "T", "sptpol_tcal_prior": "T", "sptpol_meanTcal": "1.001", "sptpol_sigmaTcal": "0.0034",
      "sptpol_pcal_prior": "T", "sptpol_kappa_prior": "T", "sptpol_alphaEE_prior": "T", "sptpol_alphaTE_prior": "T",
      "sptpol_meanAlphaTE": "-2.3"}, 4),
    ("teee_EEonly", "SPTPOL_TEEE", {"sptpol_EEonly": "T"}, 3),
    ("teee_TEonly", "SPTPOL_TEEE", {"sptpol_TEonly": "T", "correct_aberration": "T"}, 3),
    ("bb_default", "SPTPOL_BB", {}, 4),
    ("bb_priors_blind_abb", "SPTPOL_BB",
     {"sptpol_cal_prior": "T", "sptpol_invCal_90x150": "0.0001", "sptpol_Add_prior": "T", "sptpol_blind_abb": "T",
      "sptpol_blind_abb_file": "@DIR@/sptpol_blind_abb.bin"}, 4),
    ("bb_drop_90x150", "SPTPOL_BB", {"sptpol_drop_90x150ghz": "T"}, 3),
    ("bb_no_r_template", "SPTPOL_BB", {"r_template_file": ""}, 3),
]
SPTPOL_LMAX = {"SPTPOL_TEEE": 8001, "SPTPOL_BB": 2351}


def sptpol_nuisance(tag, W, seed):
    if tag == "SPTPOL_TEEE":
        g = syn.gaussians(seed, W * 11).reshape(W, 11)
        c = np.array([0.0, 0.1, 0.05, 0.1, -2.42, 0.05, -2.42, 1.0, 1.0, 0.0, 0.0])
        s = np.array([0.001, 0.02, 0.02, 0.02, 0.05, 0.01, 0.05, 0.005, 0.02, 1.0, 1.0])
        return c[None, :] + g * s[None, :]
    g = syn.gaussians(seed, W * 16).reshape(W, 16)
    c = np.array([1.0, 0.0, 0.0, 0.0132, 0.05, 0.03, 0.02, 1.0, 1.0] + [0.0] * 7)
    s = np.array([0.05, 0.01, 0.001, 0.003, 0.01, 0.01, 0.01, 0.01, 0.01] + [1.0] * 7)
    P = c[None, :] + g * s[None, :]
    P[0, 0] = 1.0            # Abb == 1: no scaling branch
    if W > 1:
        P[1, 0] = 0.0        # Abb == 0: theory zeroed
    return P


def sptpol_dataset(tag, td):
    d = os.path.join(td, tag)
    if tag == "SPTPOL_TEEE":
        return syn.make_sptpol_teee().write(d)
    return syn.make_sptpol_bb().write(d)


def gen_sptpol():
    out = {"theory_seed": 0xC05A0C, "generator": "cosmomc_amd.synthetic.make_sptpol_teee / make_sptpol_bb",
           "cases": {}}
    with tempfile.TemporaryDirectory() as td:
        paths = {t: sptpol_dataset(t, td) for t in SPTPOL_LMAX}
        for ci, (name, tag, over, W) in enumerate(SPTPOL_CASES):
            lmax = SPTPOL_LMAX[tag]
            th = syn.walker_theory(W, seed=out["theory_seed"] + 100 * ci, lmax=lmax,
                                   n_fields=3 if tag == "SPTPOL_TEEE" else 6)
            nu = sptpol_nuisance(tag, W, 5150 + ci)
            dsdir = os.path.dirname(paths[tag])
            ini = f"cmb_dataset[{tag}] = {paths[tag]}\n" + \
                "".join(f"cmb_dataset[{tag},{k}] = {v.replace('@DIR@', dsdir)}\n" for k, v in over.items())
            ref = run_cmb_harness(ini, th, nu, td)
            out["cases"][name] = {"tag": tag, "overrides": over, "walkers": W, "lmax": lmax,
                                  "theory_seed": out["theory_seed"] + 100 * ci, "nuis": nu.tolist(),
                                  "minus_lnL": ref.tolist()}
            print(f"{name:28s} -lnL = {ref}")
    with open(os.path.join(GOLDEN, "sptpol_ref.json"), "w") as f:
        json.dump(out, f, indent=1)


# TBaseParameters_SetFastSlowParams (BaseParameters.f90:302-433) through the
# compiled reference (rng_harness "blocks"): (name, config dict); likes =
# [(new_param_block_start, new_params, speed)] in the sorted list order
BLOCK_CASES = [
    ("bk15_plik_default", {"num_params": 23, "num_theory_params": 6, "varying": [1] * 6 + [1] * 8 + [0] * 9,
                           "likes": [(7, 1, 0), (8, 16, 0)]}),
    ("three_likes_shared_cal", {"num_params": 30, "num_theory_params": 6,
                                "varying": [1] * 7 + [0] * 3 + [1] * 9 + [0] * 3 + [1] * 8,
                                "likes": [(7, 1, 0), (8, 0, 0), (8, 15, 0), (23, 8, 0)]}),
    ("semi_fast_semi_slow", {"num_params": 12, "num_theory_params": 6, "index_semislow": 4, "fast_param_index": 5,
                             "varying": [1] * 12, "likes": [(7, 2, 0), (9, 4, 0)]}),
    ("no_likelihood_blocks", {"num_params": 23, "num_theory_params": 6, "varying": [1] * 14 + [0] * 9,
                              "likes": [(7, 1, 0), (8, 16, 0)], "block_fast_likelihood_params": "F"}),
    ("slow_first_likelihood", {"num_params": 20, "num_theory_params": 6, "varying": [1] * 20,
                               "likes": [(7, 3, -1), (10, 5, 0), (15, 6, 0)], "block_semi_fast": "F"}),
    ("no_fast_slow", {"num_params": 14, "num_theory_params": 6, "varying": [1] * 14, "likes": [(7, 1, 0), (8, 7, 0)],
                      "use_fast_slow": "F"}),
]


def blocks_config_text(cfg):
    lines = [f"num_params = {cfg['num_params']}", f"num_theory_params = {cfg['num_theory_params']}",
             "varying = " + " ".join(str(v) for v in cfg["varying"]), f"num_likes = {len(cfg['likes'])}"]
    lines += [f"like{i + 1} = {a} {b} {c}" for i, (a, b, c) in enumerate(cfg["likes"])]
    for k in ("index_semislow", "fast_param_index", "block_semi_fast", "block_fast_likelihood_params",
              "use_fast_slow"):
        if k in cfg:
            lines.append(f"{k} = {cfg[k]}")
    return "\n".join(lines) + "\n"


def gen_blocks():
    out = {"cases": {}}
    with tempfile.TemporaryDirectory() as td:
        for name, cfg in BLOCK_CASES:
            rows = run_rng("blocks", blocks_config_text(cfg), td)
            head = [int(x) for x in rows[0].split()]
            blocks = [[int(x) for x in r.split()][1:] for r in rows[1:1 + head[0]]]
            out["cases"][name] = {"config": cfg, "param_blocks": blocks, "num_slow": head[1], "num_fast": head[2],
                                  "num_semi_slow": head[3], "num_semi_fast": head[4]}
            print(f"{name:26s} {blocks}")
    with open(os.path.join(GOLDEN, "blocks_ref.json"), "w") as f:
        json.dump(out, f, indent=1)


# like_approx = exact on the synthetic unbinned datasets (cosmomc_amd.synthetic.make_exact):
# (name, make_exact kwargs, fields, dataset keys, hat_includes_noise, walkers, nuisance kind)
EXACT_CASES = [
    ("exact_TE_lowl", {"lmin": 2, "lmax": 29, "fksy": 1.0}, "T E", {}, False, 4, None),
    ("exact_TEB_cal_aberration", {"lmin": 2, "lmax": 400, "fksy": 0.6, "seed": 1980}, "T E B",
     {"fullsky_exact_fksy": "0.6", "calibration_param": "exact_cal.paramnames", "log_calibration_prior": "0.0025",
      "aberration_coeff": "-0.0013"}, False, 4, "cal"),
    ("exact_T_userange_hatnoise", {"lmin": 2, "lmax": 300, "fksy": 0.8, "seed": 1981}, "T",
     {"fullsky_exact_fksy": "0.8", "use_min": "10", "use_max": "250", "calibration_param": "exact_cal.paramnames"},
     True, 3, "cal"),
    ("exact_EB_pol", {"lmin": 2, "lmax": 200, "fksy": 0.5, "seed": 1982}, "E B",
     {"fullsky_exact_fksy": "0.5"}, False, 3, None),
]


def exact_dataset(case, td):
    name, kw, fields, keys, incl, W, kind = case
    return syn.make_exact(**kw).write(os.path.join(td, name), fields=fields, extra=keys, hat_includes_noise=incl)


def gen_exact():
    out = {"theory_seed": 0xE8AC7, "generator": "cosmomc_amd.synthetic.make_exact", "cases": {}}
    with tempfile.TemporaryDirectory() as td:
        for ci, case in enumerate(EXACT_CASES):
            name, kw, fields, keys, incl, W, kind = case
            path = exact_dataset(case, td)
            lmax = kw["lmax"]
            th = syn.walker_theory(W, seed=out["theory_seed"] + 100 * ci, lmax=lmax, n_fields=6)
            nu = cmbl_nuisance(kind, W, 7070 + ci) if kind else np.zeros((W, 0))
            ref = run_cmb_harness(f"cmb_dataset[exact] = {path}\n", th, nu, td)
            out["cases"][name] = {"walkers": W, "lmax": lmax, "theory_seed": out["theory_seed"] + 100 * ci,
                                  "nuis": nu.tolist(), "minus_lnL": ref.tolist()}
            print(f"{name:28s} -lnL = {ref}")
    with open(os.path.join(GOLDEN, "exact_ref.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    if not os.path.exists(os.path.join(REF_DIR, "plik_harness")):
        sys.exit("build the reference first: make -C oracle ref")
    only = sys.argv[1:]
    if not only or "plik" in only:
        gen_plik()
    if not only or "rng" in only:
        gen_rng()
    if not only or "gr" in only:
        gen_gr()
    if not only or "confid" in only:
        gen_confid()
    if not only or "cmblikes" in only:
        gen_cmblikes()
    if not only or "smica" in only:
        gen_smica()
    if not only or "sptpol" in only:
        gen_sptpol()
    if not only or "exact" in only:
        gen_exact()
    if not only or "blocks" in only:
        gen_blocks()
