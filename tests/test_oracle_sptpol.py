"""SPTpol oracle (oracle/sptpol_oracle.py) against the compiled reference
(tests/golden/sptpol_ref.json, oracle/gen_golden.py ``sptpol``): TSPTpolEELike
(CMB_SPTpol_TEEE_2017.f90) and TSPTpolBBLike (CMB_SPTpol_BB_2019.f90) on the
synthetic datasets of cosmomc_amd.synthetic, covering aberration, every prior,
the EE-only / TE-only covariance explosion, the BB drop flags, Abb = 0 / 1,
the Abb blinding offset and the r template."""
import numpy as np
import pytest

import sptpol_oracle as so
from conftest import load_golden, sptpol_overrides
from cosmomc_amd import synthetic as syn

CASES = list(load_golden("sptpol_ref.json")["cases"])


@pytest.mark.parametrize("case", CASES)
def test_sptpol_oracle_vs_reference(sptpol_golden, sptpol_data, case):
    c = sptpol_golden["cases"][case]
    ds = sptpol_data[c["tag"]]
    o = so.open_sptpol(c["tag"], ds, sptpol_overrides(c, ds))
    th = syn.walker_theory(c["walkers"], seed=c["theory_seed"], lmax=c["lmax"],
                           n_fields=3 if c["tag"] == "SPTPOL_TEEE" else 6)
    got = o.loglike_batch(th, np.array(c["nuis"]))
    np.testing.assert_allclose(got, c["minus_lnL"], rtol=1e-11, atol=1e-9)


def test_sptpol_dust_scaling_unity_at_150():
    # dustFreqScalingFrom150GHz(150, 150) == 1 (CMB_SPTpol_BB_2019.f90:799-813)
    assert abs(so.dust_scaling_from_150(150.0, 150.0) - 1.0) < 1e-15
