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


def _oracle_history(ch):
    """Every step's point and -lnL of the golden chain, replayed by the C
    oracle (pinned to the reference chain decision by decision in
    test_oracle.py)."""
    import ctypes as C

    import pyoracle as po
    from test_oracle import _target, make_oracle_proposer
    t, keep = _target(ch)
    h = make_oracle_proposer(ch)
    r = po.Ranmar(ch["ij"], ch["kl"])
    P = np.array(ch["P0"], dtype=np.float64)
    cur = C.c_double(po.lib().orc_target_loglike(C.byref(t), P))
    st = po.DragState(0, 0.0, 3.0, ch["oversample_fast"])
    Ps, likes = [], []
    for _ in range(ch["steps"]):
        if ch["fast_only"] == 2:
            po.lib().orc_drag_step(h, C.byref(r.s), C.byref(t), C.byref(st), P, C.byref(cur))
        else:
            po.lib().orc_mh_step(h, C.byref(r.s), C.byref(t), P, C.byref(cur), ch["fast_only"], None)
        Ps.append(P.copy())
        likes.append(cur.value)
    po.lib().orc_proposer_free(h)
    return np.array(Ps), np.array(likes)


CHAIN_FILE_CASES = ["gauss6_single_block", "gauss6_blocked", "gauss6_fast_only", "gauss3_n1_blocks", "gauss6_drag",
                    "gauss4_drag_every_step", "gauss27_fast21_fast_only", "gauss27_fast21_os3",
                    "gauss27_fast12_9_lincomb", "gauss40_slow_fast", "gauss27_fast21_drag"]


@pytest.mark.parametrize("name", CHAIN_FILE_CASES)
def test_chain_file_equals_reference(tmp_path, rng_golden, name):
    """ChainWriter on a golden chain's per-step history writes, byte for byte,
    the chain file the reference's own sampler wrote for it: MoveDone
    (MCMC.f90:166-190, burn_in) -> TMpiChainCollector_AddNewWeightedPoint
    (SampleCollector.f90:82-112, acc/thin weights with thin_fac = oversample_fast
    for TMetropolisSampler_GetNewSample, 1 for FastParameterSample and dragging)
    -> IO_OutputChainRow in ChainOutFile's E16.7 (settings.f90:109); and the
    same MaxLike."""
    import hashlib
    ch = rng_golden["chains"][name]
    P, like = _oracle_history(ch)
    used = np.array(ch["params_used"]) - 1
    hist = np.concatenate([P[:, used], like[:, None]], axis=1)[:, :, None]       # [steps, n_used + 1, 1]
    thin = ch["oversample_fast"] if ch["fast_only"] == 0 else 1
    assert thin == (ch["weighted_points"]["thin_fac"] or thin)
    cw = ChainWriter(str(tmp_path / "c"), [f"p{i}" for i in used], burn_in=ch["burn_in"], thin=thin)
    for a in range(0, len(like), 37):                                            # blocks of history
        cw.add_rows(hist[a:a + 37])
    cw.close()
    txt = (tmp_path / "c_1.txt").read_bytes()
    ref = ch["chain_file"]
    assert txt.count(b"\n") == ref["rows"]
    if ref["rows"]:
        assert txt.decode().splitlines()[0] == ref["first_row"]
    assert hashlib.sha256(txt).hexdigest() == ref["sha256"]
    best = cw.max_like_params(0)
    if ch["accept"][0] == 0:               # the reference's MaxLike also sees P0 when the first step accepts
        assert best[0] == pytest.approx(ch["max_like"], rel=1e-12)


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


def test_likelihood_derived_columns_and_paramnames(tmp_path):
    """Likelihood-derived parameters (addLikelihoodDerivedParams,
    GeneralTypes.f90:772-777): derived_indices from the likelihood list (derived
    names after every MCMC name, ParamNames_Add), the columns evaluated from each
    likelihood's DataParams (fixed parameters from P_fixed), written before the
    chi2 columns with '*' names."""
    import torch

    from cosmomc_amd.chains import ChainWriter, LikelihoodDerived
    from cosmomc_amd.likelihood import DataLikelihood, LikelihoodList

    class Fake(DataLikelihood):
        def __init__(self, names, dnames, fn):
            super().__init__()
            self.nuisance_names, self.derived_names, self.fn = names, dnames, fn
            self.speed = 0

        def derived_batch(self, nuis):
            return self.fn(nuis)

    a = Fake(["A1", "A2", "cal"], ["D2000"], lambda n: (n[:, 0] + n[:, 1]).reshape(-1, 1))
    b = Fake(["cal", "B"], ["Bsq", "Bcube"], lambda n: torch.stack([n[:, 1] ** 2, n[:, 1] ** 3], 1))
    a.tag, b.tag = "smica", "other"
    ll = LikelihoodList()
    ll.add(a)
    ll.add(b)
    names = ll.add_nuisance_parameters(["omegabh2"])
    assert names == ["omegabh2", "A1", "A2", "cal", "B"]
    assert a.derived_indices == [1] and b.derived_indices == [2, 3]
    P_fixed = np.array([0.0222, 30.0, 20.0, 1.0, 2.0])
    used = [2, 5]                                   # A1 and B vary; A2, cal fixed
    der = LikelihoodDerived(ll, used, P_fixed, device="cpu")
    assert [n for n, _ in der.names] == ["D2000", "Bsq", "Bcube"]
    steps, W = 3, 2
    rows = np.zeros((steps, 3, W))
    rows[:, 0, :] = 30.0 + np.arange(steps)[:, None] + np.arange(W)[None, :]
    rows[:, 1, :] = 2.0 + 0.5 * np.arange(W)[None, :]
    rows[:, 2, :] = 5.0 + np.arange(steps)[:, None]  # CurLike
    cols = der.columns(rows[:, :2, :])
    assert cols.shape == (steps, 3, W)
    np.testing.assert_array_equal(cols[:, 0, :], rows[:, 0, :] + 20.0)
    np.testing.assert_array_equal(cols[:, 1, :], rows[:, 1, :] ** 2)
    np.testing.assert_array_equal(cols[:, 2, :], rows[:, 1, :] ** 3)
    root = str(tmp_path / "c")
    cw = ChainWriter(root, ["A1", "B"], likelihoods=[a.description(), b.description()], derived=der, burn_in=0)
    cw.add_rows(rows, terms=np.ones((steps, 2, W)))
    cw.close()
    pn = [l.split("\t")[0] for l in open(root + ".paramnames").read().splitlines()]
    assert pn == ["A1", "B", "D2000*", "Bsq*", "Bcube*", "chi2_smica*", "chi2_other*", "chi2_prior*", "chi2_CMB*"]
    data = np.loadtxt(root + "_1.txt", ndmin=2)
    assert data.shape[1] == 1 + 1 + 2 + 3 + 4
