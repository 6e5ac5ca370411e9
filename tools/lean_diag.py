#!/usr/bin/env python3
"""Which (schedule, chain) variants part from the generic unpipelined chain
(mode 0, mh_body) on test_pipelined_steps_bitwise's problem, and where."""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    from cosmomc_amd import _native as N
    from cosmomc_amd import synthetic as syn
    from cosmomc_amd.likelihood import NativeCMBLikelihood
    from cosmomc_amd.sampler import BatchedMCMC
    import bench
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    calls = (1, 2, 5)
    steps = sum(calls)
    with tempfile.TemporaryDirectory() as td:
        lens_ds = os.path.join(bench.extract_refdata(td), bench.LENS_DATASET)
        data = syn.make_plik_lite(12345)
        th = syn.walker_theory(W, seed=11, n_fields=10, ld_field=2512)
        dl = torch.tensor(th, device="cuda")
        out = {}
        for mode, lean in ((0, 0), (0, 1), (1, 0), (1, 1), (3, 1), (2, 1)):
            plik = NativeCMBLikelihood("PLIK_LITE", data.write(td))
            lens = NativeCMBLikelihood("lensing", lens_ds)
            plik.nuisance_indices = [2]
            lens.nuisance_indices = [2]
            s = BatchedMCMC(W, 3, [2], [[1]], 0, [0.0222, 0.9, 3.05], [0.0222, 1.1, 3.05], [0.0, 1.0, 0.0],
                            [0.0, 0.0025, 0.0], seed_ij=61, seed_kl=72)
            s.set_covariance(np.array([[0.002 ** 2]]))
            s.add_likelihood(plik, dl)
            s.add_likelihood(lens, dl)
            assert N.lib().cmamd_debug_pipeline(s._h, mode) == 0
            assert N.lib().cmamd_debug_lean(s._h, lean) == 0
            s.enable_history(steps)
            s.set_start(np.tile([0.0222, 1.0, 3.05], (W, 1)))
            for n in calls:
                s.step(n, fast_only=True)
            out[(mode, lean)] = (s.history_host(0, steps), s.history_terms(0, steps), s.state())
            s.close()
        ref = out[(0, 0)]
        for v, o in out.items():
            dp = np.argwhere(ref[0] != o[0])
            dt = np.argwhere(ref[1] != o[1])
            print(f"mode {v[0]} lean {v[1]}: params differ at {len(dp)} (first {dp[:4].tolist()}), "
                  f"terms differ at {len(dt)} (first {dt[:4].tolist()})")
            if len(dp):
                k, i, w = dp[0]
                print("   ref", ref[0][:, :, w].T.tolist(), "\n   got", o[0][:, :, w].T.tolist())


if __name__ == "__main__":
    main()
