"""Chain-file writer (IO_OutputChainRow IO.f90:85-93, '(*(E17.7))' FileUtils.f90:75)."""
import numpy as np
import pytest

from cosmomc_amd.chains import ChainWriter, fortran_e


def test_fortran_e_format():
    assert fortran_e(1.0) == "    0.1000000E+01"
    assert fortran_e(-0.0123456789) == "   -0.1234568E-01"
    assert fortran_e(0.0) == "    0.0000000E+00"
    assert fortran_e(99999999.0) == "    0.1000000E+09"
    assert fortran_e(123.45) == "    0.1234500E+03"
    assert len(fortran_e(3.14159)) == 17


def test_run_length_rows(tmp_path):
    """Runs of identical points become one weighted row; runs crossing blocks join."""
    W, n = 2, 2
    # walker 0: A A B | B B C ; walker 1: all distinct
    pts0 = [(1.0, 5.0, 0.1), (1.0, 5.0, 0.1), (2.0, 4.0, 0.2), (2.0, 4.0, 0.2), (2.0, 4.0, 0.2), (3.0, 3.0, 0.3)]
    rows = np.zeros((6, n + 1, W))
    for t, (a, b, like) in enumerate(pts0):
        rows[t, :, 0] = [a, b, like]
        rows[t, :, 1] = [t, -t, 10.0 + t]
    cw = ChainWriter(str(tmp_path / "ch"), ["a", "b"], ranges=[(0, 10), (-1, 1)])
    cw.add_rows(rows[:3])
    cw.add_rows(rows[3:])
    cw.close()
    c0 = np.loadtxt(tmp_path / "ch_1.txt", ndmin=2)
    np.testing.assert_allclose(c0[:, 0], [2, 3, 1])               # multiplicities
    np.testing.assert_allclose(c0[:, 1], [0.1, 0.2, 0.3], rtol=1e-6)
    np.testing.assert_allclose(c0[:, 2:], [[1, 5], [2, 4], [3, 3]], rtol=1e-6)
    c1 = np.loadtxt(tmp_path / "ch_2.txt", ndmin=2)
    assert c1.shape == (6, 4) and np.all(c1[:, 0] == 1)
    assert (tmp_path / "ch.paramnames").read_text().split("\n")[0] == "a\ta"
    assert (tmp_path / "ch.ranges").exists()


def test_chi2_columns_and_likelihoods_file(tmp_path):
    """chi2_<tag> = 2 x term, chi2_prior = 2 x (like - sum terms), chi2_CMB for
    two CMB likelihoods (GeneralTypes.f90:671-776), derived names starred in
    .paramnames, 0..N ranges (ObjectParamNames.f90:480-508), .likelihoods lines
    (GeneralTypes.f90:792-812)."""
    root = str(tmp_path / "c")
    cw = ChainWriter(root, ["a"], ranges=[(0, 1)],
                     likelihoods=[("plik", "CMB", "plik_lite", "2018"), ("lens_x", "CMB", "lensing", "")])
    rows = np.zeros((3, 2, 1))
    rows[:, 0, 0] = [1.0, 1.0, 2.0]
    rows[:, 1, 0] = [10.0, 10.0, 11.0]
    terms = np.zeros((3, 2, 1))
    terms[:, 0, 0] = [4.0, 4.0, 5.0]
    terms[:, 1, 0] = [3.0, 3.0, 3.0]
    with pytest.raises(ValueError):
        cw.add_rows(rows)
    cw.add_rows(rows, terms)
    cw.close()
    c = np.loadtxt(root + "_1.txt", ndmin=2)
    np.testing.assert_allclose(c, [[2, 10, 1, 8, 6, 6, 14], [1, 11, 2, 10, 6, 6, 16]])
    pn = open(root + ".paramnames").read().splitlines()
    assert pn[1:] == ["chi2_plik*\t\\chi^2_{\\rm plik}", "chi2_lens_x*\t\\chi^2_{\\rm lens\\_x}",
                      "chi2_prior*\t\\chi^2_{\\rm prior}", "chi2_CMB*\t\\chi^2_{\\rm CMB}"]
    rg = open(root + ".ranges").read().splitlines()
    assert rg[1] == "chi2_plik".ljust(22) + "    0.0000000E+00" + "    N".ljust(17)
    assert open(root + ".likelihoods").read().splitlines() == ["1\tCMB\tplik\tplik_lite\t2018",
                                                              "1\tCMB\tlens_x\tlensing\t"]
