#!/usr/bin/env python3
"""Phase timeline of plik_quadform_ksplit (plik_lite TTTEEE, W = 1024) from
in-kernel s_memtime stamps of every workgroup (instrumented build,
tools/_stamps/, -DCMAMD_STAMPS):
  0 start, 1 first operand tiles landed, 2 K loop done, 3 partial + ticket
  done, 4 end of the last arriver's reduction, 6 partial stored and drained.
s_memtime counters are per XCD, so cross-workgroup times are compared within
one XCD only (slot 7).
Run once without arguments on the dev box (builds), then with --no-build on
the GPU."""
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
    import ctypes as C
    import tempfile

    import torch
    from cosmomc_amd import _native as N
    from cosmomc_amd import synthetic as syn
    from cosmomc_amd.likelihood import NativeCMBLikelihood
    W = int(sys.argv[sys.argv.index("--W") + 1]) if "--W" in sys.argv else 1024
    with tempfile.TemporaryDirectory() as td:
        like = NativeCMBLikelihood("PLIK_LITE", syn.make_plik_lite(12345).write(td))
        th = torch.tensor(syn.walker_theory(W, n_fields=3, ld_field=2512), device="cuda")
        cal = torch.tensor(syn.walker_calibrations(W), device="cuda").reshape(-1, 1)
        for _ in range(20):
            like.loglike_batch(th, cal)
        torch.cuda.synchronize()
        st = np.zeros((1024, 8), dtype=np.uint64)
        fn = N.lib().cmamd_debug_qf_stamps
        fn.argtypes = [C.c_void_p]
        assert fn(st.ctypes.data) == 0
    d = st.astype(np.int64)
    d = d[d[:, 0] > 0]
    print(f"workgroups {len(d)}; per-workgroup phase lengths (ticks)")
    for lab, a, b in (("first tiles", 0, 1), ("K loop", 1, 2), ("dot+partial drain", 2, 6), ("ticket", 6, 3)):
        v = d[:, b] - d[:, a]
        print(f"{lab:18s} min {v.min():7d} median {np.median(v):9.0f} max {v.max():7d}")
    last = d[d[:, 4] > 0]
    print(f"{'reduction':18s} median {np.median(last[:, 4] - last[:, 3]):9.0f}")
    for nj in sorted(set(d[:, 5])):
        m = d[:, 5] == nj
        print(f"nJ={nj}: {m.sum()} wgs, K loop median {np.median(d[m, 2] - d[m, 1]):.0f}")
    print("per XCD, relative to its first start: start / first tiles / K done / ticket done / end (max over wgs)")
    for x in sorted(set(d[:, 7])):
        e = d[d[:, 7] == x]
        t0 = e[:, 0].min()
        ends = e[e[:, 4] > 0][:, 4]
        print(f"  xcc {x}: {len(e)} wgs  start max {e[:, 0].max() - t0:6d}  first tiles med {np.median(e[:, 1] - t0):7.0f}"
              f"  K done med {np.median(e[:, 2] - t0):7.0f} max {e[:, 2].max() - t0:7d}"
              f"  ticket med {np.median(e[:, 3] - t0):7.0f} max {e[:, 3].max() - t0:7d}"
              f"  end max {(ends.max() - t0) if len(ends) else -1:7d}")
