"""Host-side checks that need no GPU: the C-ABI library loads and exports
every symbol of include/cosmomc_amd.h, argument/error handling that returns
before touching the device, ini parsing, synthetic-input determinism and the
likelihood-list bookkeeping."""
import ctypes as C
import os

import numpy as np
import pytest

from cosmomc_amd import _native as N
from cosmomc_amd import synthetic as syn
from cosmomc_amd.ini import IniFile


def test_library_exports_header_symbols():
    L = N.lib()
    syms = N.exported_symbols_from_header()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing


def test_open_missing_file_returns_error_code():
    h = C.c_void_p()
    err = C.create_string_buffer(256)
    rc = N.lib().cmbl_open(b"PLIK_LITE", b"/nonexistent/x.dataset", None, C.byref(h), err, 256)
    assert rc == -2 and b"not found" in err.value
    assert not h.value


def test_open_tag_dispatch(tmp_path):
    """CMBLikelihood_Add (CMB.f90:80-97): unknown tags are CMBlikes datasets;
    SPTpol datasets need their sptpol_* keys; SMICA is a CMBlikes dataset
    (TSmica_planck, CMBlikes.f90:1262-1339); WMAP (an external library) is not built."""
    p = tmp_path / "a.dataset"
    p.write_text("name = x\n")
    h = C.c_void_p()
    err = C.create_string_buffer(256)
    assert N.lib().cmbl_open(b"WHATEVER", str(p).encode(), None, C.byref(h), err, 256) == -3   # not a CMBlikes dataset
    assert b"fields_use" in err.value
    assert N.lib().cmbl_open(b"SPTPOL_TEEE", str(p).encode(), None, C.byref(h), err, 256) == -3
    assert b"sptpol_TEEE_params_file" in err.value
    assert N.lib().cmbl_open(b"SMICA", str(p).encode(), None, C.byref(h), err, 256) == -3   # CMBlikes ReadIni
    assert b"fields_use" in err.value
    assert N.lib().cmbl_open(b"WMAP", str(p).encode(), None, C.byref(h), err, 256) == -6


def test_sptpol_blind_r_rejected(tmp_path):
    """sptpol_blind_r needs CMB%InitPower(amp_ratio_index) (CMB_SPTpol_BB_2019.f90:585-586),
    which the batched interface does not carry: refused with CMBL_ERR_UNSUPPORTED."""
    ds = syn.make_sptpol_bb().write(str(tmp_path))
    h = C.c_void_p()
    err = C.create_string_buffer(256)
    rc = N.lib().cmbl_open(b"SPTPOL_BB", ds.encode(), b"sptpol_blind_r = T\n", C.byref(h), err, 256)
    assert rc == -6 and b"sptpol_blind_r" in err.value


def test_null_arguments_rejected():
    assert N.lib().cmbl_loglike_batch(None, 1, None, 0, 0, None, 0, None, None, None) == -1
    assert N.lib().cmbs_step(None, 1, 1, None) == -1
    assert N.lib().cmbl_open(None, None, None, None, None, 0) == -1


def test_walker_seed_mapping():
    from cosmomc_amd.sampler import walker_seed
    assert walker_seed(1802, 9373, 0) == (1802, 9373)          # walker 0 = reference chain
    seen = {walker_seed(31000, 30000, w) for w in range(2000)}
    assert len(seen) == 2000
    for ij, kl in seen:
        assert 0 <= ij <= 31328 and 0 <= kl <= 30081


def test_ini_default_include_and_overrides(tmp_path):
    (tmp_path / "base.ini").write_text("a = 1\nb = 2\n")
    (tmp_path / "inc.ini").write_text("c = 3\na = 9\n")
    (tmp_path / "main.ini").write_text("DEFAULT(base.ini)\nINCLUDE(inc.ini)\nb = 5\n"
                                       "cmb_dataset[PLIK_LITE] = %DATASETDIR%pl.dataset\n")
    ini = IniFile(str(tmp_path / "main.ini"), datasetdir=str(tmp_path) + "/")
    assert ini["b"] == "5" and ini["c"] == "3" and ini["a"] == "9"
    assert ini.relative_filename("cmb_dataset[PLIK_LITE]") == str(tmp_path) + "/pl.dataset"


def test_synthetic_is_deterministic():
    a = syn.make_plik_lite(12345)
    b = syn.make_plik_lite(12345)
    assert np.array_equal(a.X, b.X) and np.array_equal(a.cov, b.cov)
    assert a.X.size == 613 and a.cov.shape == (613, 613)
    t1 = syn.walker_theory(5, n_fields=3)
    t2 = syn.walker_theory(3, n_fields=3, first_walker=2)
    assert np.array_equal(t1[2:], t2)
    np.testing.assert_allclose(np.linalg.eigvalsh(a.cov / np.outer(np.sqrt(np.diag(a.cov)),
                                                                   np.sqrt(np.diag(a.cov))))[0], 1.0, atol=0.2)


def test_likelihood_list_nuisance_indices():
    from cosmomc_amd.likelihood import DataLikelihood, LikelihoodList
    a, b, c = DataLikelihood(), DataLikelihood(), DataLikelihood()
    a.nuisance_names, a.speed = ["calPlanck"], 5
    b.nuisance_names, b.speed = ["A_d", "A_s", "calPlanck"], -1
    c.nuisance_names, c.speed = [], 0
    L = LikelihoodList()
    for x in (a, b, c):
        L.add(x)
    names = L.add_nuisance_parameters(["omegabh2", "omegach2"])
    assert [x.speed for x in L] == [-1, 0, 5]               # sorted by speed
    assert names == ["omegabh2", "omegach2", "A_d", "A_s", "calPlanck"]
    assert b.nuisance_indices == [3, 4, 5] and a.nuisance_indices == [5]


def test_plik_dataset_written_is_readable_by_host_ini(tmp_path):
    d = syn.make_plik_lite(1)
    path = d.write(str(tmp_path))
    ini = IniFile(path)
    assert ini["use_cl"] == "TT TE EE"
    assert os.path.exists(ini.relative_filename("cov_file"))
