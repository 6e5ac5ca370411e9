#!/usr/bin/env python3
"""Run the headline bench problem for a few fast steps (no timing, no JSON):
a short program for rocprofv3 --pmc / --kernel-trace passes.

  python3 tools/probe_steps.py [--walkers W] [--steps K] [--pipe MODE] [--lib PATH]
"""
import argparse
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--walkers", type=int, default=1024)
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--pipe", type=int, default=-1, help="cmamd_debug_pipeline mode (-1: the default schedule)")
    p.add_argument("--lib", default=None, help="an instrumented libcosmomc_amd.so")
    p.add_argument("--no-lensing", action="store_true")
    a = p.parse_args()
    if a.lib:
        os.environ["COSMOMC_AMD_LIB"] = a.lib
    sys.path.insert(0, ROOT)
    import torch
    import bench
    from cosmomc_amd import _native as N
    with tempfile.TemporaryDirectory() as td:
        smp, *_ = bench.build_problem(a.walkers, 0, td, lensing=not a.no_lensing)
        if a.pipe >= 0:
            N.lib().cmamd_debug_pipeline(smp._h, a.pipe)
        smp.step(a.steps, fast_only=True)
        torch.cuda.synchronize()
    print("probe ok", a.walkers, a.steps, a.pipe)


if __name__ == "__main__":
    main()
