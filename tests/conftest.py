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


@pytest.fixture(scope="session")
def rng_golden():
    return load_golden("rng_sampler_ref.json")


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
    if os.path.isdir(os.path.join(d, "BK15")):        # configs[4]: synthetic BK15 covariance
        from cosmomc_amd import synthetic as syn
        syn.write_bk15_covmat(os.path.join(d, "BK15"))
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
