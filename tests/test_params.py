"""Parameter blocking (cosmomc_amd.params.set_fast_slow_params, a restatement
of TBaseParameters_SetFastSlowParams, BaseParameters.f90:302-433) against the
compiled reference (tests/golden/blocks_ref.json, rng_harness "blocks" mode:
the reference's own routine on BaseParams%varying and a DataLikelihoods list),
and the LikelihoodList numbering it reads (AddNuisanceParameters,
GeneralTypes.f90:618-669)."""
import json
import os
from types import SimpleNamespace

import pytest

from cosmomc_amd.params import set_fast_slow_params

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "blocks_ref.json")
with open(GOLDEN) as f:
    CASES = json.load(f)["cases"]


def _tf(v, default):
    return default if v is None else v.upper().startswith("T")


@pytest.mark.parametrize("name", sorted(CASES))
def test_blocks_vs_reference(name):
    c = CASES[name]
    cfg = c["config"]
    likes = [SimpleNamespace(new_param_block_start=a, new_params=b, speed=sp) for a, b, sp in cfg["likes"]]
    got = set_fast_slow_params(cfg["num_params"], [bool(v) for v in cfg["varying"]], likes, cfg["num_theory_params"],
                               use_fast_slow=_tf(cfg.get("use_fast_slow"), True),
                               fast_param_index=cfg.get("fast_param_index"),
                               index_semislow=cfg.get("index_semislow", -1),
                               block_semi_fast=_tf(cfg.get("block_semi_fast"), True),
                               block_fast_likelihood_params=_tf(cfg.get("block_fast_likelihood_params"), True))
    assert got.param_blocks == c["param_blocks"]
    assert (got.num_slow, got.num_fast, got.num_semi_slow, got.num_semi_fast) == \
        (c["num_slow"], c["num_fast"], c["num_semi_slow"], c["num_semi_fast"])
    assert got.slow_block_max == 2


def test_likelihood_list_numbering():
    """Sorted by speed; a shared nuisance name keeps its first index and adds
    no new parameters (ParamNames_Add skips known names); first_fast_param is
    the first fast likelihood's block start."""
    from cosmomc_amd.likelihood import DataLikelihood, LikelihoodList

    def like(names, speed):
        d = DataLikelihood()
        d.nuisance_names, d.speed = names, speed
        return d
    L = LikelihoodList()
    bk, lens, plik = like(["BBdust", "BBsync"], 0), like(["calPlanck"], 0), like(["calPlanck"], -1)
    for x in (bk, lens, plik):
        L.add(x)
    names = L.add_nuisance_parameters(["omegabh2", "omegach2"])
    assert names == ["omegabh2", "omegach2", "calPlanck", "BBdust", "BBsync"]
    assert [x for x in L] == [plik, bk, lens]
    assert (plik.new_param_block_start, plik.new_params, plik.nuisance_indices) == (3, 1, [3])
    assert (bk.new_param_block_start, bk.new_params, bk.nuisance_indices) == (4, 2, [4, 5])
    assert (lens.new_param_block_start, lens.new_params, lens.nuisance_indices) == (6, 0, [3])
    assert L.first_fast_param == 4
