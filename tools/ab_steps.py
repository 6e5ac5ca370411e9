#!/usr/bin/env python3
"""Interleaved A/B of fast-step variants on the headline problem (W = 1024,
plik_lite TTTEEE + lensing): every variant is a (pipeline mode, lean chain)
pair set through the debug switches; each repetition times every variant's
K steps (bench.py's barrier-free single-GPU timing: synchronize, K steps,
synchronize) and then its per-kernel HIP-event averages.

  python3 tools/ab_steps.py [--steps K] [--reps R] [--variants 1:1,1:0,3:1,3:0]
"""
import argparse
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--walkers", type=int, default=1024)
    p.add_argument("--steps", type=int, default=300)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--variants", default="1:1,1:0,3:1,3:0", help="mode:lean pairs")
    a = p.parse_args()
    sys.path.insert(0, ROOT)
    import torch
    import bench
    from cosmomc_amd import _native as N
    variants = [tuple(int(x) for x in v.split(":")) for v in a.variants.split(",")]
    with tempfile.TemporaryDirectory() as td:
        runs = {}
        for v in variants:
            smp, *_ = bench.build_problem(a.walkers, 0, td)
            assert N.lib().cmamd_debug_pipeline(smp._h, v[0]) == 0
            assert N.lib().cmamd_debug_lean(smp._h, v[1]) == 0
            smp.step(a.warmup, fast_only=True)
            runs[v] = smp
        torch.cuda.synchronize()
        for r in range(a.reps):
            for v, smp in runs.items():
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                smp.step(a.steps, fast_only=True)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                kern = bench.kernel_profile(smp, a.steps)
                print(f"rep {r} mode {v[0]} lean {v[1]}: {a.walkers * a.steps / dt / 1e6:7.3f} M evals/s "
                      f"{dt / a.steps * 1e6:6.2f} us/step  {kern}", flush=True)
        # the chains agree across variants
        st = [smp.state() for smp in runs.values()]
        import numpy as np
        same = all(np.array_equal(st[0][0], s[0]) and np.array_equal(st[0][1], s[1]) for s in st[1:])
        print("states identical across variants:", same)


if __name__ == "__main__":
    main()
