"""Importance sampling host logic (cosmomc_amd/importance.py, reference
TImportanceSampler_ImportanceSample, ImportanceSampling.f90:105-411) with an
analytic GetLogLikePost; the GPU evaluator is covered in
tests/test_gpu_importance.py."""
import math

import numpy as np
import pytest

from cosmomc_amd.chains import fortran_e
from cosmomc_amd.importance import ImportanceSampler, ImportanceSettings, LOGZERO, read_chain_rows


def _write_chain(path, rows):
    with open(path, "w") as f:
        for r in rows:
            f.write("".join(fortran_e(v) for v in r) + "\n")


def _chain(n=40, seed=3):
    rng = np.random.default_rng(seed)
    x = rng.normal(size=(n, 2))
    like = 0.5 * np.sum(x ** 2, axis=1)
    mult = rng.integers(1, 5, size=n).astype(float)
    return np.column_stack([mult, like, x])


def _eval(P):       # new target: shifted Gaussian in the two used parameters, bound |x| < 3
    t = 0.5 * np.sum((P[:, :2] - 0.3) ** 2, axis=1)
    t[np.any(np.abs(P[:, :2]) > 3, axis=1)] = LOGZERO
    return t


class _BoundedEval:
    """_eval with the new run's hard bounds exposed as prior_cut (GPUEvaluator does the same)."""

    def __call__(self, P):
        return _eval(P)

    def prior_cut(self, P):
        return np.any(np.abs(P[:, :2]) > 3, axis=1)


def test_prior_cut_rows_skipped_before_counting(tmp_path):
    """A row outside the new prior bounds is skipped before anything is
    counted (CheckPriorCuts, ImportanceSampling.f90:296-302): it adds nothing
    to num_used, mult_ratio or weight_min."""
    rows = _chain()
    rows[5, 2] = 3.5
    _write_chain(tmp_path / "in.txt", rows)
    st = ImportanceSettings(redo_likelihoods=True, redo_skip=0, redo_auto_likescale=False)
    r = ImportanceSampler(st, [1, 2], np.zeros(3), _BoundedEval()).run(str(tmp_path / "in.txt"))
    chain = read_chain_rows(str(tmp_path / "in.txt"))
    inside = ~np.any(np.abs(chain[:, 2:4]) > 3, axis=1)
    assert not inside[5]
    chain = chain[inside]
    tl = _eval(np.column_stack([chain[:, 2:], np.zeros(len(chain))]))
    w = np.exp(chain[:, 1] - tl)
    assert r.num_used == inside.sum()
    assert r.mult_ratio == pytest.approx(w.sum())
    assert r.weight_min == pytest.approx(w.min()) and r.weight_min > 0
    assert len(r.rows) == inside.sum()


def test_nint_rounds_half_away_from_zero(tmp_path):
    """redo_skip fraction x lines = 2.5 -> NINT 3 (ImportanceSampling.f90:147-148),
    where Python's round would give 2."""
    from cosmomc_amd.importance import nint
    assert nint(2.5) == 3 and nint(3.5) == 4 and nint(-2.5) == -3 and nint(2.4999) == 2
    rows = _chain(10)
    _write_chain(tmp_path / "in.txt", rows)
    st = ImportanceSettings(redo_likelihoods=False, redo_skip=0.25)
    mult, like, P = ImportanceSampler(st, [1, 2], np.zeros(2), _eval).read(str(tmp_path / "in.txt"))
    assert mult.size == 10 - 3


def test_weights_and_rows(tmp_path):
    rows = _chain()
    rows[5, 2] = 3.5                      # an evaluator without prior_cut: weight 0, row dropped
    _write_chain(tmp_path / "in.txt", rows)
    st = ImportanceSettings(redo_likelihoods=True, redo_skip=0, redo_auto_likescale=False)
    r = ImportanceSampler(st, [1, 2], np.zeros(3), _eval).run(str(tmp_path / "in.txt"), str(tmp_path / "post"))
    chain = read_chain_rows(str(tmp_path / "in.txt"))       # E17.7 rounded input
    tl = _eval(np.column_stack([chain[:, 2:], np.zeros(len(chain))]))
    w = np.where(tl == LOGZERO, 0.0, np.exp(chain[:, 1] - tl))
    keep = chain[:, 0] * w > 1e-100
    out = read_chain_rows(str(tmp_path / "post.txt"))
    assert out.shape[0] == keep.sum() and not keep[5] and keep.sum() >= rows.shape[0] - 3
    np.testing.assert_allclose(out[:, 0], (chain[:, 0] * w)[keep], rtol=1e-6)
    np.testing.assert_allclose(out[:, 1], tl[keep], rtol=1e-6)
    assert r.num_used == rows.shape[0]
    assert r.mult_ratio == pytest.approx(w.sum())
    assert r.weight_min == 0.0
    assert r.effective_samples == pytest.approx((chain[:, 0] * w).sum() / (chain[:, 0] * w).max())
    # rows go through the reference's ChainOutFile format, E16.7 (settings.f90:109,
    # ImportanceSampling.f90:221 -> WriteParams), byte for byte as the chain writer's
    from cosmomc_amd.chains import fortran_e
    with open(tmp_path / "post.txt") as f:
        lines = f.read().splitlines()
    for line, (m, t, pu) in zip(lines, r.rows):
        assert line == "".join(fortran_e(v, 16) for v in [m, t, *pu])
        assert len(line) == 16 * (2 + len(pu))


def test_skip_thin_and_fraction(tmp_path):
    rows = _chain(30)
    rows[:, 0] = 2.0
    _write_chain(tmp_path / "in.txt", rows)
    st = ImportanceSettings(redo_likelihoods=False, redo_skip=4, redo_thin=3)
    s = ImportanceSampler(st, [1, 2], np.zeros(2), _eval)
    mult, like, P = s.read(str(tmp_path / "in.txt"))
    # 26 rows of weight 2 thinned by 3 (:279-289)
    acc, expect = 0, []
    for _ in range(26):
        acc += 2
        if acc >= 3:
            expect.append(acc // 3)
            acc %= 3
    assert list(mult) == expect
    st2 = ImportanceSettings(redo_likelihoods=False, redo_skip=0.5)
    m2, _, _ = ImportanceSampler(st2, [1, 2], np.zeros(2), _eval).read(str(tmp_path / "in.txt"))
    assert m2.size == 15                  # nint(lines * 0.5) skipped (:146-148)


def test_auto_likescale_restart(tmp_path):
    """A likelihood offset > redo_max_logLike_diff after redo_auto_likescale_count
    rows restarts with redo_likeoffset = max_truelike - max_like (:340-362)."""
    rows = _chain(20)
    _write_chain(tmp_path / "in.txt", rows)

    def far(P):
        return _eval(P) + 50.0
    st = ImportanceSettings(redo_likelihoods=True, redo_skip=0)
    r = ImportanceSampler(st, [1, 2], np.zeros(2), far).run(str(tmp_path / "in.txt"))
    chain = read_chain_rows(str(tmp_path / "in.txt"))
    tl = far(chain[:, 2:])
    off = tl[:5].min() - chain[:5, 1].min()
    assert r.likeoffset == pytest.approx(off)
    w = np.exp(chain[:, 1] - tl + off)
    assert r.mult_ratio == pytest.approx(w.sum())
    assert 0.01 < r.mean_weight < 100


def test_nochange_and_change_like_only(tmp_path):
    rows = _chain(10)
    _write_chain(tmp_path / "in.txt", rows)
    chain = read_chain_rows(str(tmp_path / "in.txt"))
    for key in ("redo_nochange", "redo_change_like_only"):
        st = ImportanceSettings(redo_likelihoods=True, redo_skip=0, redo_auto_likescale=False, **{key: True})
        r = ImportanceSampler(st, [1, 2], np.zeros(2), _eval).run(str(tmp_path / "in.txt"))
        np.testing.assert_allclose([m for m, _, _ in r.rows], chain[:, 0])
        tl = [t for _, t, _ in r.rows]
        if key == "redo_nochange":
            np.testing.assert_allclose(tl, chain[:, 1])
        else:
            np.testing.assert_allclose(tl, _eval(chain[:, 2:]))


def test_settings_from_ini():
    ini = {"redo_likelihoods": "T", "redo_theory": "F", "redo_skip": "0.3", "redo_thin": "2",
           "redo_temp": "2.5", "redo_likeoffset": "1d0", "redo_auto_likescale": "F"}
    s = ImportanceSettings.from_ini(ini)
    assert s.redo_likelihoods and not s.redo_theory and s.redo_thin == 2
    assert s.redo_skip == 0.3 and s.redo_temp == 2.5 and s.redo_likeoffset == 1.0 and not s.redo_auto_likescale
    with pytest.raises(ValueError):
        ImportanceSettings.from_ini({"redo_add": "T"})
    assert math.isclose(ImportanceSettings().redo_max_logLike_diff, 10.0)
