import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu")


def load_golden(name):
    import json
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def plik_golden():
    return load_golden("plik_lite_ref.json")


def expand_chain(ch):
    """A sampler golden chain with its test problem rebuilt from the seed
    (cosmomc_amd.synthetic.chain_problem; the fixture stores only the
    reference's results and checksums of the problem it ran on).  Adds cov,
    center, bounds, priors, P0 and linear_combinations, the per-step accept
    list, and at[k] = the index of step k in the stored rows (P, cur_like,
    trial_like) or None."""
    import numpy as np

    import gen_golden as gg
    from cosmomc_amd import synthetic as syn
    prob = syn.chain_problem(ch["n"], ch["problem_seed"], ch["extra"])
    np.testing.assert_allclose(gg.problem_sums(prob), ch["problem_sums"], rtol=1e-15, atol=0,
                               err_msg="rebuilt chain problem differs from the one the reference ran on")
    cov, center, pmin, pmax, pmean, pstd, P0, lin = prob
    ch = dict(ch, cov=cov.tolist(), center=center.tolist(), pmin=pmin.tolist(), pmax=pmax.tolist(),
              prior_mean=pmean.tolist(), prior_std=pstd.tolist(), P0=P0.tolist(), linear_combinations=lin)
    ch["accept"] = [int(c) for c in ch["accept"]]
    pos = {k: i for i, k in enumerate(ch["stored_steps"])}
    ch["at"] = [pos.get(k) for k in range(ch["steps"])]
    return ch


@pytest.fixture(scope="session")
def rng_golden():
    g = load_golden("rng_sampler_ref.json")
    g["chains"] = {k: expand_chain(v) for k, v in g["chains"].items()}
    return g


@pytest.fixture(scope="session")
def gr_golden():
    return load_golden("gr_ref.json")


@pytest.fixture(scope="session")
def cmbl_golden():
    return load_golden("cmblikes_ref.json")


@pytest.fixture(scope="session")
def refdata(tmp_path_factory):
    """The reference's own CMBlikes data files (tests/golden/refdata.tar.xz,
    packed by oracle/pack_refdata.py) extracted to a temporary directory."""
    import io
    import lzma
    import tarfile
    d = str(tmp_path_factory.mktemp("refdata"))
    with open(os.path.join(GOLDEN, "refdata.tar.xz"), "rb") as f:
        tar = tarfile.open(fileobj=io.BytesIO(lzma.decompress(f.read())))
        try:
            tar.extractall(d, filter="data")
        except TypeError:
            tar.extractall(d)
    from cosmomc_amd import synthetic as syn
    syn.write_refdata_extras(d)                       # configs[4]'s BK15 covariance, bk_cal.paramnames
    return d


@pytest.fixture(scope="session")
def sptpol_golden():
    return load_golden("sptpol_ref.json")


@pytest.fixture(scope="session")
def sptpol_data(tmp_path_factory):
    """The synthetic SPTpol TEEE / BB datasets (cosmomc_amd.synthetic) written
    once per session: {tag: dataset path}."""
    from cosmomc_amd import synthetic as syn
    d = str(tmp_path_factory.mktemp("sptpol"))
    return {"SPTPOL_TEEE": syn.make_sptpol_teee().write(os.path.join(d, "SPTPOL_TEEE")),
            "SPTPOL_BB": syn.make_sptpol_bb().write(os.path.join(d, "SPTPOL_BB"))}


def sptpol_overrides(case, dataset):
    """Golden-case overrides with @DIR@ -> the dataset's directory."""
    d = os.path.dirname(dataset)
    return {k: v.replace("@DIR@", d) for k, v in case["overrides"].items()}


@pytest.fixture(scope="session")
def exact_golden():
    return load_golden("exact_ref.json")


@pytest.fixture(scope="session")
def exact_data(tmp_path_factory):
    """The synthetic unbinned like_approx = exact datasets of oracle/gen_golden.py
    EXACT_CASES, written once per session: {case name: dataset path}."""
    import gen_golden as gg
    d = str(tmp_path_factory.mktemp("exact"))
    return {c[0]: gg.exact_dataset(c, d) for c in gg.EXACT_CASES}


@pytest.fixture(scope="session")
def smica_golden():
    return load_golden("smica_ref.json")


@pytest.fixture(scope="session")
def smica_data(tmp_path_factory):
    """The synthetic SMICA datasets (cosmomc_amd.synthetic.make_smica), gaussian
    and HL, written once per session: {like_approx: dataset path}."""
    from cosmomc_amd import synthetic as syn
    d = str(tmp_path_factory.mktemp("smica"))
    data = syn.make_smica()
    return {a: data.write(os.path.join(d, a), like_approx=a) for a in ("gaussian", "HL")}
