#!/usr/bin/env python3
"""Repeated CMBlikes / SPTpol loglike_batch calls for kernel profiling
(rocprofv3) and per-dataset throughput.

    python tools/cmbl_profile.py [lensing|bk|spt|bk15|sptteee|sptbb] [W] [iters]
"""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from cosmomc_amd import _native as N  # noqa: E402
from cosmomc_amd import synthetic as syn  # noqa: E402
from cosmomc_amd.likelihood import NativeCMBLikelihood  # noqa: E402

CASES = {"lensing": ("lensing", bench.LENS_DATASET, {}, 2500, 1),
         "bk": ("BKPLANCK", "BKPlanck/BKPlanck_detset_comb_dust.dataset", {}, 600, 16),
         "spt": ("SPT", "sptsz_2500d_tt/spt_s13_margfg.dataset", {}, 3300, 1),
         "bk15": ("BKPLANCK", "BK15/BK15_dust.dataset",
                  {"maps_use": "BK15_95_B BK15_150_B BK15_220_B W023_B P030_B W033_B P044_B P070_B P100_B "
                               "P143_B P217_B P353_B"}, 600, 16),
         "sptteee": ("SPTPOL_TEEE", None, {}, 8001, 11),
         "sptbb": ("SPTPOL_BB", None, {}, 2351, 16)}
BK_FID = [3.0, 1.0, -0.42, 1.59, 19.6, -0.6, -3.3, 0.1, 2.0, 1.0, 1.0, 1.0, 0.0, 0.0, 0.0, 0.0]
SPT_FID = {"sptteee": [0.0, 0.1, 0.05, 0.1, -2.42, 0.05, -2.42, 1.0, 1.0, 0.0, 0.0],
           "sptbb": [1.0, 0.0, 0.0, 0.0132, 0.05, 0.03, 0.02, 1.0, 1.0] + [0.0] * 7}

if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "lensing"
    W = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    tag, ds, over, lmax, nn = CASES[which]
    with tempfile.TemporaryDirectory() as td:
        if which == "sptteee":
            path = syn.make_sptpol_teee().write(td)
        elif which == "sptbb":
            path = syn.make_sptpol_bb().write(td)
        else:
            rd = bench.extract_refdata(td)
            if which == "bk15":
                syn.write_bk15_covmat(os.path.join(rd, "BK15"))
            path = os.path.join(rd, ds)
        like = NativeCMBLikelihood(tag, path, over)
        nf = {"sptteee": 3, "sptbb": 6}.get(which, 10)
        th = torch.tensor(syn.walker_theory(W, lmax=lmax, ld_field=lmax + 1 + (lmax + 1) % 2, n_fields=nf),
                          device="cuda")
        nu = np.ones((W, nn))
        if which in ("bk", "bk15"):
            nu[:] = BK_FID
        if which in SPT_FID:
            nu[:] = SPT_FID[which]
        nu = torch.tensor(nu, device="cuda")
        ws = torch.empty(like.workspace_bytes(W), dtype=torch.uint8, device="cuda")
        out = torch.empty(W, dtype=torch.float64, device="cuda")
        for _ in range(3):
            like.loglike_batch(th, nu, out, ws)
        torch.cuda.synchronize()
        N.profile_reset()
        N.profile_enable(True)
        for _ in range(iters):
            like.loglike_batch(th, nu, out, ws)
        torch.cuda.synchronize()
        N.profile_enable(False)
        for k in ("cmbl_bk_prologue", "cmbl_window_kernel", "cmbl_reduce_kernel", "cmbl_gauss_small_kernel",
                  "cmbl_hl_kernel", "cmbl_quadform", "sptpol_window_kernel", "sptpol_delta_kernel",
                  "sptpol_quadform"):
            t, n = N.profile_read(k)
            if n:
                print(f"{which} W={W} {k:22s} {t / n * 1e3:9.2f} us")
        torch.cuda.synchronize()
        import time
        t0 = time.perf_counter()
        for _ in range(iters):
            like.loglike_batch(th, nu, out, ws)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / iters
        print(f"{which} W={W} total {dt * 1e6:9.2f} us/call  {W / dt / 1e6:8.3f} M evals/s")
