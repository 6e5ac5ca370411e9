#!/usr/bin/env python3
"""Fixed cost of one cmbs_step call on the headline problem: for K fast steps
per call, the host time until cmbs_step returns (the launches enqueued) and
the wall time until the stream is idle, medians over repeated calls.  The
intercept of wall time against K is the per-call cost the driver's 20-step
command pays once (host work before the first launch, the first and last
launches' difference from a middle one, the final synchronisation).
"""
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if __name__ == "__main__":
    import torch

    import bench
    reps = int(os.environ.get("REPS", "30"))
    with tempfile.TemporaryDirectory() as td:
        smp, *_ = bench.build_problem(1024, 0, td)
        smp.step(20, fast_only=True)
        torch.cuda.synchronize()
        rows = []
        for K in (1, 2, 5, 10, 20, 50):
            host, wall = [], []
            for _ in range(reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                smp.step(K, fast_only=True)
                t1 = time.perf_counter()
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                host.append(t1 - t0)
                wall.append(t2 - t0)
            rows.append((K, 1e6 * np.median(host), 1e6 * np.median(wall)))
            print(f"K={K:3d}  host {rows[-1][1]:8.1f} us  wall {rows[-1][2]:8.1f} us  "
                  f"({rows[-1][2] / K:6.2f} us/step)", flush=True)
        k = np.array([r[0] for r in rows], dtype=float)
        w = np.array([r[2] for r in rows])
        slope, icpt = np.polyfit(k, w, 1)
        print(f"fit: wall = {icpt:.1f} us + {slope:.2f} us x K")
        # an empty stream round trip, for scale
        e = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            torch.cuda.synchronize()
            e.append(time.perf_counter() - t0)
        print(f"idle synchronize: {1e6 * np.median(e):.1f} us")
