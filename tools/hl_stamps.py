#!/usr/bin/env python3
"""Per-phase cycles of the first Jacobi rounds of cmbl_hl_rows_kernel (block 0,
lane 0) from in-kernel s_memtime stamps, on the BK15 dataset at W = 1024.

Builds an instrumented copy of the library (tools/_stamps/, -DCMAMD_STAMPS):
  0->1 pair + diagonal exchange, 1->2 (c, s), 2->3 column rotation,
  3->4 row rotation, 4->0' loop back.
"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tools", "_stamps")
if __name__ == "__main__":
    if "--no-build" not in sys.argv:
        subprocess.run(["make", "-C", os.path.join(ROOT, "cosmomc_amd", "csrc"), "-j8", f"OUT={OUT}",
                        "EXTRA=-DCMAMD_STAMPS"], check=True, stdout=subprocess.DEVNULL)
        sys.exit(0)
    os.environ["COSMOMC_AMD_LIB"] = os.path.join(OUT, "libcosmomc_amd.so")
    sys.path.insert(0, ROOT)
    import runpy
    sys.argv = [os.path.join(ROOT, "tools", "cmbl_profile.py"), "bk15", "1024", "3"]
    runpy.run_path(sys.argv[0], run_name="__main__")
    from cosmomc_amd import _native as N
    st = np.zeros((32, 6), dtype=np.uint64)
    assert N.lib().cmamd_debug_hl_stamps(st.ctypes.data_as(C.c_void_p)) == 0
    d = st.astype(np.int64)
    names = ["pair+diag exch", "(c, s)", "column rot", "row rot"]
    for i, n in enumerate(names):
        print(f"{n:16s} median {np.median(d[:, i + 1] - d[:, i]):8.0f}  max {(d[:, i + 1] - d[:, i]).max():8.0f}")
    print(f"{'round':16s} median {np.median(d[1:, 0] - d[:-1, 0]):8.0f} (s_memtime ticks)")
    sw = np.zeros((2, 64), dtype=np.uint32)
    assert N.lib().cmamd_debug_hl_sweeps(sw.ctypes.data_as(C.c_void_p)) == 0
    for k, lab in enumerate(("first eigensolve", "second eigensolve")):
        h = sw[k]
        nz = np.nonzero(h)[0]
        print(f"{lab}: waves by sweeps (incl. the final check sweep) " +
              " ".join(f"{i}:{h[i]}" for i in nz) + f"  mean {(h * np.arange(64)).sum() / max(h.sum(), 1):.2f}")
