#!/usr/bin/env python3
"""Single-core timing of the REFERENCE's own LogLike (oracle/_ref/plik_bench,
compiled from /root/reference by oracle/Makefile) on the datasets the GPU
profiles cover, for the per-dataset comparison in DESIGN.md.  Development
container only (the reference never travels to the GPU box).

    python tools/ref_cpu_timing.py [seconds]
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from cosmomc_amd import synthetic as syn  # noqa: E402
import gen_golden as gg  # noqa: E402

BK15_MAPS = gg.BK15_MAPS


def bench(ini_text, theory, nuis, td, seconds):
    W, nf, nl = theory.shape
    ini = os.path.join(td, "b.ini")
    with open(ini, "w") as f:
        f.write(ini_text)
    th, nu = os.path.join(td, "th.bin"), os.path.join(td, "nu.bin")
    np.ascontiguousarray(theory, dtype="<f8").tofile(th)
    np.ascontiguousarray(nuis, dtype="<f8").tofile(nu)
    env = dict(os.environ, OPENBLAS_NUM_THREADS="1", OMP_NUM_THREADS="1")
    out = subprocess.run([os.path.join(ROOT, "oracle", "_ref", "plik_bench"), ini, th, nu, str(W), str(nl - 1),
                          str(nf), str(nuis.shape[1]), str(seconds)], check=True, cwd=td, env=env,
                         capture_output=True, text=True).stdout.split()[-3:]
    n, t = float(out[0]), float(out[1])
    return n / t


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
    W = 16
    rows = []
    with tempfile.TemporaryDirectory() as td:
        ds = syn.make_sptpol_teee().write(os.path.join(td, "teee"))
        rows.append(("SPTPOL_TEEE (synthetic, 56 bins x 2, l 50..8000)",
                     bench(f"cmb_dataset[SPTPOL_TEEE] = {ds}\n", syn.walker_theory(W, lmax=8001, n_fields=3),
                           gg.sptpol_nuisance("SPTPOL_TEEE", W, 1), td, secs)))
        ds = syn.make_sptpol_bb().write(os.path.join(td, "bb"))
        rows.append(("SPTPOL_BB (synthetic, 7 bins x 3, l 50..2350)",
                     bench(f"cmb_dataset[SPTPOL_BB] = {ds}\n", syn.walker_theory(W, lmax=2351, n_fields=6),
                           gg.sptpol_nuisance("SPTPOL_BB", W, 2), td, secs)))
        rd = gg.refdata_dir(td)
        bk = os.path.join(rd, gg.BK15)
        nu = gg.cmbl_nuisance("bk_sync", W, 3)
        rows.append(("BK15 B-only 12 maps x 9 bins (HL)",
                     bench(f"cmb_dataset[BKPLANCK] = {bk}\ncmb_dataset[BKPLANCK,maps_use] = {BK15_MAPS}\n",
                           syn.walker_theory(W, lmax=600), nu, td, secs)))
        bkp = os.path.join(rd, gg.BKP)
        rows.append(("BKPlanck 10 maps x 9 bins (HL)",
                     bench(f"cmb_dataset[BKPLANCK] = {bkp}\n", syn.walker_theory(W, lmax=600),
                           gg.cmbl_nuisance("bk_sync", W, 4), td, secs)))
    print("reference LogLike, amdflang -O2 + OpenBLAS, 1 thread, dev container CPU:")
    for name, r in rows:
        print(f"  {name:52s} {r:12.1f} evals/s  ({1e6 / r:9.1f} us/eval)")


if __name__ == "__main__":
    main()
