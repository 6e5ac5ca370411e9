#!/usr/bin/env python3
"""Run the bench's config4_fast21 workload for a few dozen fast steps (no
convergence leg), for a rocprofv3 --kernel-trace of per-launch durations:
    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c4 -o run -- python3 tools/c4_trace.py
then  python3 tools/c4_trace.py --summary gpurun_out/c4/run_kernel_trace.csv"""
import csv
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if len(sys.argv) > 2 and sys.argv[1] == "--summary":
    import collections
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(sys.argv[2])):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("cmamd::", "")
        d[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    for k, v in d.items():
        v2 = sorted(v)
        print(f"{k:40s} n={len(v):5d} min {v2[0]:8.2f} median {v2[len(v) // 2]:8.2f} max {v2[-1]:8.2f} "
              f"mean {sum(v) / len(v):8.2f}")
        if "rot" in k or "mh" in k:
            print("   first 46:", " ".join(f"{x:.1f}" for x in v[:46]))
    sys.exit(0)

import bench  # noqa: E402

if os.environ.get("C4_STAGE_R"):            # debug: rotation rows staged (1) or read in place (0)
    from cosmomc_amd import _native as N
    from cosmomc_amd.sampler import BatchedMCMC
    _orig = BatchedMCMC.set_covariance

    def _patched(self, cov):
        _orig(self, cov)
        assert N.lib().cmamd_debug_stage_R(self._h, int(os.environ["C4_STAGE_R"])) == 0
    BatchedMCMC.set_covariance = _patched
with tempfile.TemporaryDirectory() as td:
    print(bench.config4_run(512, 0, 1, td, -1, steps=42))
