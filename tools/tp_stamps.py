#!/usr/bin/env python3
"""Block timeline of theory_window_kernel (the fused window pass) from
in-kernel s_memtime stamps: per XCD the span of its blocks, per item the
block durations (prologue, step loop, epilogue) against its steps and active
MFMA blocks.  Builds the instrumented library (tools/_stamps/,
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
        st = np.zeros((4096, 10), dtype=np.uint64)
        assert N.lib().cmamd_debug_tp_stamps(st.ctypes.data_as(C.c_void_p)) == 0
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.save(os.path.join(ROOT, "gpurun_out", "tp_stamps.npy"), st)
    used = np.nonzero(st[:, 3])[0]
    s = st[used].astype(np.int64)
    hw, xcc, item, work = s[:, 4], s[:, 5] & 15, s[:, 6], s[:, 7]
    cu = (hw >> 8) & 15
    se = (hw >> 13) & 7
    print(f"blocks {len(used)}, items {len(np.unique(item))}")
    for x in np.unique(xcc):
        m = xcc == x
        t0 = s[m, 0].min()
        print(f"XCC {x}: blocks {m.sum():4d} span {s[m, 3].max() - t0:7d}  start skew {s[m, 0].max() - t0:7d}"
              f"  last start {s[m, 0].max() - t0:7d}  CUs used {len(np.unique(se[m] * 16 + cu[m]))}")
    print("item  steps actblk  blocks  prologue  loop  epilogue  total (median cycles)")
    for it in np.unique(item):
        m = item == it
        pr, lo, ep = s[m, 1] - s[m, 0], s[m, 2] - s[m, 1], s[m, 3] - s[m, 2]
        print(f"{it:4d} {work[m][0] // 1000:6d} {work[m][0] % 1000:6d} {m.sum():7d} {np.median(pr):9.0f} "
              f"{np.median(lo):6.0f} {np.median(ep):9.0f} {np.median(s[m, 3] - s[m, 0]):6.0f}")
