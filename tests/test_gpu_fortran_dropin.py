"""The Fortran drop-in of INTEGRATION.md section 2, end to end: the
NativeCMB module (extracted from INTEGRATION.md and compiled by
`make -C oracle native` against the reference's own modules) evaluates
plik_lite TTTEEE and Planck 2018 lensing through TNativeCMBLike%LogLike ->
cmbl_loglike_batch_host (W = 1 per call), driven like the reference harness;
the values must equal the compiled reference's own LogLike goldens.
GPU only; skipped when the binary was not built (no /root/reference when the
tree was built)."""
import os
import subprocess

import numpy as np
import pytest

from cosmomc_amd import synthetic as syn

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "oracle", "_ref", "native_check")


def _run(tmp_path, tag, dataset, theory, nuis):
    W, nfield, nl = theory.shape
    th, nu, out = (str(tmp_path / x) for x in ("th.bin", "nu.bin", "out.txt"))
    np.ascontiguousarray(theory, dtype="<f8").tofile(th)
    np.ascontiguousarray(nuis, dtype="<f8").tofile(nu)
    subprocess.run([EXE, tag, dataset, th, nu, str(W), str(nl - 1), str(nfield), str(nuis.shape[1]), out],
                   check=True, timeout=120, cwd=str(tmp_path))
    return np.loadtxt(out, ndmin=1)


@pytest.mark.skipif(not os.path.exists(EXE), reason="oracle/_ref/native_check not built")
def test_fortran_dropin_plik_lite(plik_golden, tmp_path):
    c = plik_golden["cases"]["plik_lite_TTTEEE"]
    ds = syn.make_plik_lite(plik_golden["data_seed"]).write(str(tmp_path / "plik"))
    th = syn.walker_theory(c["walkers"], seed=plik_golden["theory_seed"], n_fields=3)
    got = _run(tmp_path, "PLIK_LITE", ds, th, np.array(c["cal"])[:, None])
    np.testing.assert_allclose(got, c["minus_lnL"], rtol=1e-10, atol=0)


@pytest.mark.skipif(not os.path.exists(EXE), reason="oracle/_ref/native_check not built")
def test_fortran_dropin_lensing(cmbl_golden, refdata, tmp_path):
    c = cmbl_golden["cases"]["lensing_consext8"]
    th = syn.walker_theory(c["walkers"], seed=c["theory_seed"], lmax=c["lmax"])
    got = _run(tmp_path, c["tag"], os.path.join(refdata, c["dataset"]), th, np.array(c["nuis"]))
    np.testing.assert_allclose(got, c["minus_lnL"], rtol=1e-10, atol=1e-9)
