#!/usr/bin/env python3
"""Phase timing of mh_kernel<accept, propose> from in-kernel s_memtime stamps.

Builds an instrumented copy of the library (tools/_stamps/, -DCMAMD_STAMPS),
runs the bench problem and prints the median cycles of each phase:
  0->1 issue LDS-DMA, 1->2 wait DMA, 2->3 accept, 3->4 propose + nuisance
  scatter, 4->5 write-back issue, 5->6 store drain.
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
                        "EXTRA=-DCMAMD_STAMPS " + os.environ.get("STAMP_EXTRA", "")], check=True,
                       stdout=subprocess.DEVNULL)
    os.environ["COSMOMC_AMD_LIB"] = os.path.join(OUT, "libcosmomc_amd.so")
    sys.path.insert(0, ROOT)
    import torch
    import bench
    from cosmomc_amd import _native as N
    W = int(os.environ.get("W", "1024"))
    with tempfile.TemporaryDirectory() as td:
        smp, *_ = bench.build_problem(W, 0, td)
        # the unpipelined steps: mh_kernel's workgroups are the first 64 of
        # their launch (in the unified launch they come last, past the stamps)
        assert N.lib().cmamd_debug_pipeline(smp._h, 0) == 0
        smp.step(20, fast_only=True)
        torch.cuda.synchronize()
        st = np.zeros((64, 16), dtype=np.uint64)
        assert N.lib().cmamd_debug_stamps(st.ctypes.data_as(C.c_void_p)) == 0
    nb = min(64, (W + 63) // 64)
    d = np.diff(st[:nb, :7].astype(np.int64), axis=1)
    names = ["dma issue", "dma wait", "accept", "propose", "writeback issue", "store drain"]
    for i, n in enumerate(names):
        print(f"{n:16s} median {np.median(d[:, i]):8.0f}  max {d[:, i].max():8.0f} cycles")
    fine = [("accept: mask/terms", 2, 8), ("accept: target_like", 8, 9), ("accept: randexp", 9, 10),
            ("accept: move", 10, 11), ("accept: history", 11, 3), ("propose->map done", 4, 12),
            ("scatter + sync", 12, 13), ("writeback", 13, 5)]
    for n, a, b in fine:
        if st[:nb, a].any() and st[:nb, b].any():
            dd = st[:nb, b].astype(np.int64) - st[:nb, a].astype(np.int64)
            print(f"{n:20s} median {np.median(dd):8.0f}  max {dd.max():8.0f} cycles")
    tot = st[:nb, 6].astype(np.int64) - st[:nb, 0].astype(np.int64)
    print(f"{'total':16s} median {np.median(tot):8.0f}  max {tot.max():8.0f}")
    print("block start skew (cycles):", int(st[:nb, 0].max() - st[:nb, 0].min()))
