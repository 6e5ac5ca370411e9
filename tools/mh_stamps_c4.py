#!/usr/bin/env python3
"""mh_kernel phase cycles, step by step, on the config4_fast21 workload
(one 21-parameter fast block: a new 21x21 random rotation every 21 steps per
walker).  Same instrumented build as tools/mh_stamps.py (run that first on
the dev box to build tools/_stamps/); then on the GPU:
    python tools/mh_stamps_c4.py
Phases: 0->1 issue LDS-DMA, 1->2 wait, 2->3 accept, 3->4 propose, 4->5
write-back issue, 5->6 drain.  Each mh launch of a step overwrites the stamps,
so one step is run per read (the accept+propose launch is the last)."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["COSMOMC_AMD_LIB"] = os.path.join(os.environ.get("STAMP_OUT", os.path.join(ROOT, "tools", "_stamps")), "libcosmomc_amd.so")
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from cosmomc_amd import _native as N  # noqa: E402
from cosmomc_amd.sampler import BatchedMCMC  # noqa: E402

n, W = 21, 512
rng = np.random.default_rng(2121)
width = rng.uniform(0.05, 2.0, n)
A = rng.standard_normal((n, n))
cov = (A @ A.T / n + np.eye(n)) * np.outer(width, width) / 2
P0 = rng.uniform(-1.0, 1.0, n)
used = list(range(1, n + 1))
smp = BatchedMCMC(W, n, used, [used], 0, P0 - 20 * width, P0 + 20 * width, propose_scale=2.4, seed_ij=4004,
                  seed_kl=9373)
smp.set_covariance(np.diag(width ** 2))
smp.set_test_gaussian(cov, P0)
if os.environ.get("C4_STAGE_R"):     # force the rotation rows staged (1) or in HBM (0)
    assert N.lib().cmamd_debug_stage_R(smp._h, int(os.environ["C4_STAGE_R"])) == 0
smp.set_start(np.tile(P0, (W, 1)))
rows = []
for step in range(44):
    smp.step(2, fast_only=True)        # one accept+propose launch (the stamped one) per call
    torch.cuda.synchronize()
    st = np.zeros((64, 16), dtype=np.uint64)
    assert N.lib().cmamd_debug_stamps(st.ctypes.data_as(C.c_void_p)) == 0
    d = np.diff(st[:W // 16, :7].astype(np.int64), axis=1)   # 16-walker blocks
    fine = [(2, 8), (8, 9), (9, 10), (10, 11), (11, 3), (3, 14), (14, 15), (15, 4), (4, 12), (12, 13), (13, 5)]
    f = [np.median(st[:W // 16, b].astype(np.int64) - st[:W // 16, a].astype(np.int64)) if st[:W // 16, b].any()
         else 0 for a, b in fine]
    rows.append(np.concatenate([np.median(d, axis=0), f]))
rows = np.array(rows)
rt = np.zeros(3, dtype=np.uint64)
fn = N.lib().cmamd_debug_rot_ticks
fn.argtypes = [C.c_void_p]
assert fn(rt.ctypes.data) == 0
print(f"rot_kernel first listed walker, last rotation: total {rt[0]} ticks, Gaussian draws {rt[1]}, Gram-Schmidt {rt[2]}")
names = ["dma issue", "dma wait", "accept", "propose", "wb issue", "drain", "a:terms", "a:target", "a:randexp",
         "a:move", "a:hist", "p:copy", "p:prop", "p:post", "p:map", "p:scatter", "p:wb"]
print("step  " + " ".join(f"{x:>9s}" for x in names))
for i, r in enumerate(rows):
    print(f"{i:4d}  " + " ".join(f"{v:9.0f}" for v in r))
