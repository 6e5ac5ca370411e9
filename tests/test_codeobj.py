"""The built library's gfx950 kernels, read from their code-object metadata on
the CPU (tools/codeobj.py): no hot kernel keeps a copy of its arguments in
scratch.  A kernel that indexes its by-value configuration with a run-time
index, or calls a non-inlined function on it, gets a per-lane scratch copy of
it (1 KB and more for DevCfg), which makes every lane's loads and stores go to
memory -- round 5 measured the Metropolis + window-pass launch at 66 us instead of
24 us that way."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
LIB = os.path.join(ROOT, "cosmomc_amd", "lib", "libcosmomc_amd.so")

HOT = ("mh_kernel", "mh_bin_kernel", "mh_step_kernel", "quadform", "theory_window",
       "cmbl_window", "cmbl_hl", "cmbl_gauss_small", "plik_", "sptpol_", "drag_", "rot_kernel")


@pytest.fixture(scope="module")
def kernels():
    if not os.path.exists(LIB):
        pytest.skip("libcosmomc_amd.so not built (make -C cosmomc_amd/csrc)")
    import codeobj
    return codeobj.kernels(LIB)


def test_every_kernel_present(kernels):
    names = " ".join(kernels)
    for k in ("mh_step_kernel", "mh_kernel", "quadform_corun", "theory_window_vec", "cmbl_hl_rows_kernel",
              "rot_kernel", "mh_bin_kernel", "sptpol_window_kernel"):
        assert k in names, k


def test_no_argument_copy_in_scratch(kernels):
    hot = {n: k for n, k in kernels.items() if any(h in n for h in HOT)}
    assert len(hot) > 20
    big = {n: k["scratch"] for n, k in hot.items() if k["scratch"] > 256}
    assert not big, big
    mh = {n: k["scratch"] for n, k in hot.items() if "mh_" in n and k["scratch"] > 64}
    assert not mh, mh
