#!/usr/bin/env python3
"""Block timeline of the unified step launch (mh_step_kernel) from in-kernel
s_memrealtime stamps (100 MHz): per role (quadratic form, chi^2, pass,
Metropolis) when its workgroups start and end, and for the Metropolis
workgroups when their tile's wait ends.  Builds the instrumented library
(tools/_stamps/ or STAMP_OUT, -DCMAMD_STAMPS) unless --no-build, then runs 20
headline fast steps and reports the last middle launch.
"""
import ctypes as C
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.environ.get("STAMP_OUT", os.path.join(ROOT, "tools", "_stamps"))
ROLES = {1: "quadform", 2: "chi2", 3: "pass", 4: "metropolis"}

if __name__ == "__main__":
    if "--no-build" not in sys.argv:
        subprocess.run(["make", "-C", os.path.join(ROOT, "cosmomc_amd", "csrc"), "-j8", f"OUT={OUT}",
                        "EXTRA=-DCMAMD_STAMPS"], check=True, stdout=subprocess.DEVNULL)
        sys.exit(0)
    os.environ["COSMOMC_AMD_LIB"] = os.path.join(OUT, "libcosmomc_amd.so")
    sys.path.insert(0, ROOT)
    import torch
    import bench
    from cosmomc_amd import _native as N
    q = lambda a: " ".join(f"{np.percentile(a, p):6.2f}" for p in (0, 10, 50, 90, 100))
    with tempfile.TemporaryDirectory() as td:
        smp, *_ = bench.build_problem(1024, 0, td)
        smp.step(20, fast_only=True)
        torch.cuda.synchronize()
        st2 = np.zeros((2, 2048, 6), dtype=np.uint64)
        assert N.lib().cmamd_debug_uni_stamps(st2.ctypes.data_as(C.c_void_p)) == 0
    for which, st in (("a middle launch", st2[0]), ("the last (accept-only) launch", st2[1])):
        s = st[st[:, 4] > 0].astype(np.int64)
        t0 = s[:, 0].min()
        us = lambda x: (x - t0) / 100.0
        print(f"{which} ({os.environ.get('CMAMD_TAIL_ORDER', 'default order')}): quantiles 0/10/50/90/100, "
              f"us from the first block's start; launch {us(s[:, 3].max()):.2f} us")
        for r, name in ROLES.items():
            b = s[s[:, 4] == r]
            if not len(b):
                continue
            print(f"  {name:10s} {len(b):4d}  start {q(us(b[:, 0]))}   end {q(us(b[:, 3]))}   "
                  f"dur {q((b[:, 3] - b[:, 0]) / 100.0)}")
            if r == 4:
                if (b[:, 5] > 0).all():
                    print(f"  {'':10s}       folded chi^2 done {q(us(b[:, 5]))}")
                print(f"  {'':10s}       wait done {q(us(b[:, 1]))}")
