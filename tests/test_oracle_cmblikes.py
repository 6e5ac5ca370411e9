"""CMBlikes oracle (oracle/cmblikes_oracle.py) against the compiled reference
(tests/golden/cmblikes_ref.json) on the reference's own datasets: Planck 2018
lensing (gaussian + linear correction + calPlanck), BICEP2/Keck/Planck (HL +
foregrounds, decorrelation), SPT-SZ (aberration + log-calibration prior), BK15
(12 B maps x 9 bins, band-centre errors; synthetic covariance, the one file the
reference does not ship)."""
import os

import numpy as np
import pytest

import cmblikes_oracle as co
from cosmomc_amd import synthetic as syn

CASES = ["lensing_consext8", "bkplanck_3map_bins1to5", "bkplanck_all_maps", "bkplanck_decorr_lin_quad",
         "bkplanck_EB_4map", "sptsz_aberration_calprior", "bk15_B_12maps", "bk15_B_decorr_bandcentre",
         "bkplanck_calparam_prior"]


@pytest.mark.parametrize("case", CASES)
def test_cmblikes_oracle_vs_reference(cmbl_golden, refdata, case):
    c = cmbl_golden["cases"][case]
    o = co.CMBLikesOracle(os.path.join(refdata, c["dataset"]), c["overrides"], c["tag"])
    th = syn.walker_theory(c["walkers"], seed=c["theory_seed"], lmax=c["lmax"])
    nu = np.array(c["nuis"])
    got = np.array([o.loglike(th[w], nu[w]) for w in range(c["walkers"])])
    np.testing.assert_allclose(got, c["minus_lnL"], rtol=1e-11, atol=1e-9)


EXACT = ["exact_TE_lowl", "exact_TEB_cal_aberration", "exact_T_userange_hatnoise", "exact_EB_pol"]


@pytest.mark.parametrize("case", EXACT)
def test_exact_oracle_vs_reference(exact_golden, exact_data, case):
    """like_approx = exact (ExactChiSq, CMBlikes.f90:967-979) on the synthetic
    unbinned datasets vs the compiled reference (tests/golden/exact_ref.json)."""
    c = exact_golden["cases"][case]
    o = co.CMBLikesOracle(exact_data[case], None, "exact")
    th = syn.walker_theory(c["walkers"], seed=c["theory_seed"], lmax=c["lmax"], n_fields=6)
    nu = np.array(c["nuis"]).reshape(c["walkers"], -1)
    got = np.array([o.loglike(th[w], nu[w]) for w in range(c["walkers"])])
    np.testing.assert_allclose(got, c["minus_lnL"], rtol=1e-11, atol=1e-9)


SMICA = ["smica_gauss", "smica_gauss_run", "smica_gauss_calname", "smica_hl_aber_calname", "smica_calparam_override",
         "smica_calname_unknown"]


@pytest.mark.parametrize("case", SMICA)
def test_smica_oracle_vs_reference(smica_golden, smica_data, case):
    """TSmica_planck (CMBlikes.f90:1262-1339): the TT foreground, nuisance_params,
    calibration_paramname (and the base calibration_param it overrides) and the
    derived D_l(2000), against the compiled reference (tests/golden/smica_ref.json)."""
    c = smica_golden["cases"][case]
    o = co.CMBLikesOracle(smica_data[c["like_approx"]], c["overrides"], "SMICA")
    th = syn.walker_theory(c["walkers"], seed=c["theory_seed"], lmax=c["lmax"], n_fields=6)
    nu = np.array(c["nuis"])
    got = np.array([o.loglike(th[w], nu[w]) for w in range(c["walkers"])])
    np.testing.assert_allclose(got, c["minus_lnL"], rtol=1e-11, atol=1e-9)
    der = np.array([o.derived(nu[w]) for w in range(c["walkers"])])
    np.testing.assert_allclose(der, np.array(c["derived"]), rtol=1e-14, atol=0)
    assert o.derived_names == ["Dl2000_smica"]
