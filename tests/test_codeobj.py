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


def test_asm_loads_waited_before_use(tmp_path):
    """The unified launch's quadratic form loads the raw sums with inline asm
    and waits for them with a hand-counted vmcnt (qfs_body.h): rebuild
    sampler.hip's gfx950 assembly and check that no instruction reads, copies
    or reuses a load's registers before a wait covers it
    (tools/check_asm_loads.py; a dead prefetch's registers once became MFMA
    accumulators while the load was in flight)."""
    import shutil
    import subprocess
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    src = os.path.join(ROOT, "cosmomc_amd", "csrc")
    out = str(tmp_path / "sampler.s")
    subprocess.run([hipcc, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=off", "-x", "hip",
                    "-S", "sampler.hip", "-o", out, "--offload-device-only"], cwd=src, check=True,
                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_asm_loads.py"), out],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:]
    last = r.stdout.strip().splitlines()[-1]
    assert last.endswith("0 bad, 0 to review") and int(last.split()[0]) > 0, r.stdout[-2000:]
