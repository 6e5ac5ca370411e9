#!/usr/bin/env python3
"""Repeated CMBlikes loglike_batch calls for kernel profiling (rocprofv3).

    python tools/cmbl_profile.py [lensing|bk|spt] [W] [iters]
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
         "spt": ("SPT", "sptsz_2500d_tt/spt_s13_margfg.dataset", {}, 3300, 1)}

if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "lensing"
    W = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    tag, ds, over, lmax, nn = CASES[which]
    with tempfile.TemporaryDirectory() as td:
        like = NativeCMBLikelihood(tag, os.path.join(bench.extract_refdata(td), ds), over)
        th = torch.tensor(syn.walker_theory(W, lmax=lmax, ld_field=lmax + 1 + (lmax + 1) % 2), device="cuda")
        nu = np.ones((W, nn))
        if which == "bk":
            nu[:] = [3.0, 1.0, -0.42, 1.59, 19.6, -0.6, -3.3, 0.1, 2.0, 1.0, 1.0, 1.0, 0.0, 0.0, 0.0, 0.0]
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
                  "cmbl_hl_kernel", "cmbl_quadform"):
            t, n = N.profile_read(k)
            if n:
                print(f"{k:22s} {t / n * 1e3:9.2f} us")
