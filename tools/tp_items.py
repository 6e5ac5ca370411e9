#!/usr/bin/env python3
"""The fused window pass's work items at the headline workload (field, l range,
32-l steps, columns, 16-column blocks), from cmamd_debug_tp_items."""
import ctypes as C
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from cosmomc_amd import _native as N  # noqa: E402

with tempfile.TemporaryDirectory() as td:
    smp, *_ = bench.build_problem(1024, 0, td)
    out = np.zeros(6 * 256, dtype=np.int32)
    n = N.lib().cmamd_debug_tp_items(smp._h, out.ctypes.data_as(C.c_void_p), 256)
    print("items", n)
    tot = 0
    for k in range(n):
        f, l0, l1, st, nc, nb = out[6 * k:6 * k + 6]
        tot += st
        print(f"{k:3d} field {f} l {l0:5d}-{l1:5d} ({l1 - l0 + 1:4d} l) steps {st:2d} cols {nc:2d} blocks {nb}")
    print("steps per tile", tot)
