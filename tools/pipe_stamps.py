#!/usr/bin/env python3
"""Block timeline of mh_pass_kernel (the pipelined fast steps: the Metropolis
workgroups and the fused window pass in one launch) from in-kernel
s_memrealtime stamps (100 MHz): when the Metropolis blocks end, when the pass
blocks finish streaming, how long they wait for their tile's calibrations,
and when they end.  Builds the instrumented library (tools/_stamps/,
-DCMAMD_STAMPS) unless --no-build, then runs 20 headline fast steps.
"""
import ctypes as C
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.environ.get("STAMP_OUT", os.path.join(ROOT, "tools", "_stamps"))
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
    with tempfile.TemporaryDirectory() as td:
        smp, *_ = bench.build_problem(1024, 0, td)
        smp.step(20, fast_only=True)
        torch.cuda.synchronize()
        st = np.zeros((2048, 5), dtype=np.uint64)
        assert N.lib().cmamd_debug_pipe_stamps(st.ctypes.data_as(C.c_void_p)) == 0
    s = st[st[:, 4] > 0].astype(np.int64)
    t0 = s[:, 0].min()
    us = lambda x: (x - t0) / 100.0
    mh, ps = s[s[:, 4] == 1], s[s[:, 4] == 2]
    q = lambda a: " ".join(f"{np.percentile(a, p):6.2f}" for p in (0, 10, 50, 90, 100))
    print("quantiles 0/10/50/90/100, us from the first block's start")
    print(f"mh   blocks {len(mh):4d}  start {q(us(mh[:, 0]))}  end {q(us(mh[:, 3]))}")
    print(f"pass blocks {len(ps):4d}  start {q(us(ps[:, 0]))}")
    print(f"      streamed  {q(us(ps[:, 1]))}")
    print(f"      wait done {q(us(ps[:, 2]))}")
    print(f"      end       {q(us(ps[:, 3]))}")
    print(f"      waited    {q((ps[:, 2] - ps[:, 1]) / 100.0)}")
