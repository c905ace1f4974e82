"""scann_amd.scann_builder emits the same config as the reference builder
(fixtures: tests/golden/builder_configs.json, made by
tests/golden/make_builder_configs.py from the reference's scann_builder.py)."""
import json
import math
import os

import numpy as np
import pytest

from scann_amd import scann_builder
from scann_amd.config import parse_text_proto, search_config_from_text

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "builder_configs.json")
CASES = json.load(open(GOLDEN))


def _norm(tree):
    """Parsed text proto -> comparable (NaN-safe, bool/enum normalised)."""
    if isinstance(tree, dict):
        return {k: [_norm(v) for v in vs] for k, vs in sorted(tree.items())}
    if isinstance(tree, float) and math.isnan(tree):
        return "nan"
    if isinstance(tree, bool):
        return str(tree).lower()
    if isinstance(tree, str) and tree.lower() in ("true", "false"):
        return tree.lower()
    return tree


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_builder_mirror_matches_reference_config(case):
    b = scann_builder.ScannBuilder(np.zeros(case["shape"], np.float32), case["num_neighbors"],
                                   case["distance"])
    for meth, kw in case["calls"]:
        b = getattr(b, meth)(**kw)
    mine = _norm(parse_text_proto(b.create_config()))
    ref = _norm(parse_text_proto(case["config"]))
    assert mine == ref


def test_reference_glove_config_interpreted():
    case = next(c for c in CASES if c["name"] == "glove_tree_ah")
    cfg = search_config_from_text(case["config"])
    assert (cfg.metric, cfg.num_leaves, cfg.leaves_to_search) == ("dot_product", 1000, 100)
    assert cfg.dims_per_block == 2 and cfg.residual and cfg.reorder_num_neighbors == 100
    assert cfg.num_neighbors == 10 and cfg.soar_lambda is None


def test_reference_soar_and_l2_configs_interpreted():
    soar = search_config_from_text(next(c for c in CASES if c["name"] == "dot96_soar")["config"])
    assert soar.soar_lambda == 1.5 and soar.overretrieve_factor == 2.0
    l2 = search_config_from_text(next(c for c in CASES if c["name"] == "sift_l2")["config"])
    assert l2.metric == "squared_l2" and not l2.residual


@pytest.mark.parametrize("name", ["brute_force", "lut256_l2"])
def test_unsupported_configs_rejected(name):
    with pytest.raises(ValueError):
        search_config_from_text(next(c for c in CASES if c["name"] == name)["config"])


def test_builder_errors_mirror_reference():
    b = scann_builder.ScannBuilder(np.zeros((10, 8), np.float32), 5, "dot_product")
    b.tree(4, 2)
    with pytest.raises(Exception, match="already been configured"):
        b.tree(4, 2)
    with pytest.raises(ValueError, match="Exactly 1 of score_ah"):
        b.create_config()
    with pytest.raises(ValueError, match="distance_measure must be one of"):
        scann_builder.ScannBuilder(np.zeros((10, 8)), 5, "cosine").score_ah(2).create_config()
    with pytest.raises(ValueError, match="SOAR requires dot product"):
        scann_builder.ScannBuilder(np.zeros((10, 8)), 5, "squared_l2").tree(
            4, 2, soar_lambda=1.5).score_ah(2).create_config()
    with pytest.raises(Exception, match="no builder lambda"):
        scann_builder.ScannBuilder(np.zeros((10, 8)), 5, "dot_product").tree(4, 2).score_ah(2).build()


def test_config_parser_is_strict():
    with pytest.raises(ValueError):
        parse_text_proto("num_neighbors: 10 partitioning { num_children: 3")
    with pytest.raises(ValueError):
        parse_text_proto("a: }")
