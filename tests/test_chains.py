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
    """Runs of identical points become one weighted row; runs crossing blocks
    join; the point a chain sits at when the run ends is not written."""
    W, n = 2, 2
    # walker 0: A A B | B B C ; walker 1: all distinct
    pts0 = [(1.0, 5.0, 0.1), (1.0, 5.0, 0.1), (2.0, 4.0, 0.2), (2.0, 4.0, 0.2), (2.0, 4.0, 0.2), (3.0, 3.0, 0.3)]
    rows = np.zeros((6, n + 1, W))
    for t, (a, b, like) in enumerate(pts0):
        rows[t, :, 0] = [a, b, like]
        rows[t, :, 1] = [t, -t, 10.0 + t]
    cw = ChainWriter(str(tmp_path / "ch"), ["a", "b"], ranges=[(0, 10), (-1, 1)], burn_in=-1)
    cw.add_rows(rows[:3])
    cw.add_rows(rows[3:])
    cw.close()
    c0 = np.loadtxt(tmp_path / "ch_1.txt", ndmin=2)
    np.testing.assert_allclose(c0[:, 0], [2, 3])                  # multiplicities
    np.testing.assert_allclose(c0[:, 1], [0.1, 0.2], rtol=1e-6)
    np.testing.assert_allclose(c0[:, 2:], [[1, 5], [2, 4]], rtol=1e-6)
    c1 = np.loadtxt(tmp_path / "ch_2.txt", ndmin=2)
    assert c1.shape == (5, 4) and np.all(c1[:, 0] == 1)
    assert (tmp_path / "ch.paramnames").read_text().split("\n")[0] == "a\ta"
    assert (tmp_path / "ch.ranges").exists()


def test_chi2_columns_and_likelihoods_file(tmp_path):
    """chi2_<tag> = 2 x term, chi2_prior = 2 x (like - sum terms), chi2_CMB for
    two CMB likelihoods (GeneralTypes.f90:671-776), derived names starred in
    .paramnames, 0..N ranges (ObjectParamNames.f90:480-508), .likelihoods lines
    (GeneralTypes.f90:792-812)."""
    root = str(tmp_path / "c")
    cw = ChainWriter(root, ["a"], ranges=[(0, 1)],
                     likelihoods=[("plik", "CMB", "plik_lite", "2018"), ("lens_x", "CMB", "lensing", "")], burn_in=-1)
    rows = np.zeros((4, 2, 1))
    rows[:, 0, 0] = [1.0, 1.0, 2.0, 3.0]
    rows[:, 1, 0] = [10.0, 10.0, 11.0, 12.0]
    terms = np.zeros((4, 2, 1))
    terms[:, 0, 0] = [4.0, 4.0, 5.0, 5.0]
    terms[:, 1, 0] = [3.0, 3.0, 3.0, 3.0]
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


@pytest.mark.parametrize("name,burn_in,thin", [("gauss6_blocked", 2, 2), ("gauss3_n1_blocks", 2, 3),
                                               ("gauss6_fast_only", 0, 1), ("gauss27_fast21_os3", 5, 3)])
def test_rows_follow_movedone_restatement(tmp_path, rng_golden, name, burn_in, thin):
    """ChainWriter on a reference chain's per-step history (the golden's points
    and -lnL after every step) writes exactly the rows the event-by-event
    MoveDone / AddNewWeightedPoint restatement (oracle) writes for its accept
    sequence: burn_in drops the first burn_in + 1 stays, thin = oversample_fast
    turns multiplicities into acc/thin weights."""
    import pyoracle as po
    ch = rng_golden["chains"][name]
    P, like = np.array(ch["P"]), np.array(ch["cur_like"])
    used = np.array(ch.get("params_used", range(1, ch["n"] + 1))) - 1
    hist = np.concatenate([P[:, used], like[:, None]], axis=1)[:, :, None]       # [steps, n_used + 1, 1]
    cw = ChainWriter(str(tmp_path / "c"), [f"p{i}" for i in used], burn_in=burn_in, thin=thin)
    for a in range(0, len(like), 37):                                            # blocks of history
        cw.add_rows(hist[a:a + 37])
    cw.close()
    ref, (ml, mp) = po.move_done_rows(ch["like0"], ch["P0"], ch["accept"], like, P, burn_in, thin)
    got = np.loadtxt(str(tmp_path / "c_1.txt"), ndmin=2)
    ref = np.array(ref)[:, [0, 1] + [2 + i for i in used]]
    assert got.shape == ref.shape and len(ref) > 10
    np.testing.assert_allclose(got, ref, rtol=1e-6, atol=1e-12)                  # E17.7 text
    best, pts = cw.max_like_params(0)
    assert best == ml
    np.testing.assert_allclose(pts[1:], np.asarray(mp)[used])


def test_weights_thin_and_burn(tmp_path):
    """Hand case: stays of length 5, 1, 2, 4, 3 with burn_in 1, thin 3: the
    first two stays are dropped, then acc 2 -> no row, acc 6 -> weight 2,
    acc 3 -> weight 1 (SampleCollector.f90:97-104)."""
    lens = [5, 1, 2, 4, 3, 1]
    rows = []
    for i, L in enumerate(lens):
        rows += [[float(i), 10.0 + i]] * L
    cw = ChainWriter(str(tmp_path / "h"), ["x"], burn_in=1, thin=3)
    cw.add_rows(np.array(rows)[:, :, None])
    cw.close()
    c = np.loadtxt(str(tmp_path / "h_1.txt"), ndmin=2)
    np.testing.assert_allclose(c, [[2.0, 13.0, 3.0], [1.0, 14.0, 4.0]])
