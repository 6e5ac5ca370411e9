#!/usr/bin/env python3
"""Jacobi sweep counts of cmbl_hl_rows_kernel's two eigensolves (waves by the
number of sweeps, from the instrumented build's counters) on the BK15 dataset
at W = 1024, after tools/cmbl_profile.py's per-dataset profile.  Builds an
instrumented copy of the library (tools/_stamps/, -DCMAMD_STAMPS) first.
"""
import ctypes as C
import os
import subprocess
import sys

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
    import runpy
    sys.argv = [os.path.join(ROOT, "tools", "cmbl_profile.py"), "bk15", "1024", "3"]
    runpy.run_path(sys.argv[0], run_name="__main__")
    from cosmomc_amd import _native as N
    sw = np.zeros((2, 64), dtype=np.uint32)
    assert N.lib().cmamd_debug_hl_sweeps(sw.ctypes.data_as(C.c_void_p)) == 0
    for k, lab in enumerate(("first eigensolve", "second eigensolve")):
        h = sw[k]
        nz = np.nonzero(h)[0]
        print(f"{lab}: waves by sweeps (incl. the final check sweep) " +
              " ".join(f"{i}:{h[i]}" for i in nz) + f"  mean {(h * np.arange(64)).sum() / max(h.sum(), 1):.2f}")
    ph = np.zeros(4, dtype=np.uint64)
    assert N.lib().cmamd_debug_hl_phase(ph.ctypes.data_as(C.c_void_p)) == 0
    n = max(int(ph[3]), 1)
    print(f"Jacobi rounds (lane 0 of every wave): {n}; s_memtime ticks per round: "
          f"write+barrier {ph[0] / n:.0f}, read+dot+angle {ph[1] / n:.0f}, rotate+barrier {ph[2] / n:.0f}, "
          f"total {(ph[0] + ph[1] + ph[2]) / n:.0f}")
    tp = np.zeros(12, dtype=np.uint64)
    assert N.lib().cmamd_debug_hl_tp(tp.ctypes.data_as(C.c_void_p)) == 0
    nw = max(int(tp[11]), 1)
    names = ["loads", "to_basis 1", "solve 1", "from_basis 1 + U rows + T = Chat U, R (2)", "Rot = U R U^T (3)",
             "to_basis 2", "solve 2", "from_basis 2 + g(x) + V rows (4)", "(5) + output"]
    print(f"kernel phases, s_memtime ticks per wave (lane 0 of {nw} waves):")
    for i, nm in enumerate(names):
        print(f"   {nm:45s} {tp[i] / nw:9.0f}")
