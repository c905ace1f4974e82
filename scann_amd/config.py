"""Minimal reader for the ScannConfig text protos the builder emits.

The reference parses its config with protobuf TextFormat and, notably,
IGNORES parse errors (scann/scann_ops/cc/scann.h:182-188).  This reader is
strict instead: a malformed config raises ValueError.

Only the fields the tree-AH LUT16 query path needs are interpreted
(``SearchConfig`` below); everything else is kept in the tree and ignored.
"""
from __future__ import annotations

import dataclasses
import re
from typing import Any, Dict, List, Optional

_TOKEN = re.compile(r'\s*(?:(#[^\n]*)|([{}:])|("(?:[^"\\]|\\.)*")|([^\s{}:"#]+))')


def _tokens(text: str):
    pos = 0
    while pos < len(text):
        m = _TOKEN.match(text, pos)
        if not m or m.end() == pos:
            if text[pos:].strip() == "":
                return
            raise ValueError(f"config parse error near: {text[pos:pos + 40]!r}")
        pos = m.end()
        if m.group(1) is not None:
            continue
        tok = m.group(2) or m.group(3) or m.group(4)
        if tok is not None:
            yield tok


def _scalar(tok: str) -> Any:
    if tok.startswith('"'):
        return bytes(tok[1:-1], "utf-8").decode("unicode_escape")
    low = tok.lower()
    if low in ("true", "false"):
        return low == "true"
    if low in ("nan", "-nan"):
        return float("nan")
    if low in ("inf", "infinity"):
        return float("inf")
    try:
        return int(tok)
    except ValueError:
        pass
    try:
        return float(tok)
    except ValueError:
        return tok  # enum value


def parse_text_proto(text: str) -> Dict[str, List[Any]]:
    """Parse into {field: [values]} where message values are nested dicts."""
    toks = list(_tokens(text))
    pos = 0

    def message(end_brace: bool):
        nonlocal pos
        out: Dict[str, List[Any]] = {}
        while pos < len(toks):
            t = toks[pos]
            if t == "}":
                if not end_brace:
                    raise ValueError("unbalanced '}' in config")
                pos += 1
                return out
            name = t
            pos += 1
            if pos < len(toks) and toks[pos] == ":":
                pos += 1
            if pos >= len(toks):
                raise ValueError(f"missing value for field {name!r}")
            if toks[pos] == "{":
                pos += 1
                val = message(True)
            else:
                if toks[pos] in ("{", "}", ":"):
                    raise ValueError(f"bad value for field {name!r}")
                val = _scalar(toks[pos])
                pos += 1
            out.setdefault(name, []).append(val)
        if end_brace:
            raise ValueError("unbalanced '{' in config")
        return out

    return message(False)


def _get(tree: Optional[Dict[str, List[Any]]], *path, default=None):
    cur: Any = tree
    for p in path:
        if not isinstance(cur, dict) or p not in cur:
            return default
        cur = cur[p][0]
    return cur


@dataclasses.dataclass
class SearchConfig:
    """What the MI355X tree-AH searcher needs from a ScannConfig."""

    num_neighbors: int
    metric: str                       # "dot_product" | "squared_l2"
    num_leaves: int
    leaves_to_search: int
    training_iterations: int = 12
    training_sample_size: int = 100000
    dims_per_block: int = 2
    residual: bool = True
    ah_training_iterations: int = 10
    ah_training_sample_size: int = 100000
    reorder_num_neighbors: Optional[int] = None
    soar_lambda: Optional[float] = None
    overretrieve_factor: float = 2.0
    noise_shaping_threshold: Optional[float] = None   # AVQ; None / NaN = plain encoding
    raw: Optional[Dict[str, List[Any]]] = None

    @property
    def has_reordering(self) -> bool:
        return self.reorder_num_neighbors is not None


_DISTANCES = {"DotProductDistance": "dot_product", "SquaredL2Distance": "squared_l2"}


def _noise_shaping(ah) -> Optional[float]:
    """AsymmetricHasherConfig.noise_shaping_threshold (NaN = off).  Noise-shaped
    training of the codebooks (use_noise_shaped_training) is not implemented
    and is rejected rather than ignored."""
    if _get(ah, "use_noise_shaped_training"):
        raise ValueError("use_noise_shaped_training is not supported (AVQ applies to the "
                         "encoding; the codebooks are trained by plain k-means)")
    t = _get(ah, "noise_shaping_threshold")
    if t is None:
        return None
    t = float(t)
    return None if t != t else t


def search_config_from_text(text: str) -> SearchConfig:
    return search_config_from_tree(parse_text_proto(text))


def search_config_from_tree(tree: Dict[str, List[Any]]) -> SearchConfig:
    """SearchConfig of a parsed config: a text proto (parse_text_proto) or a
    binary scann_config.pb decoded by scann_amd.assets."""
    nn = _get(tree, "num_neighbors")
    if nn is None:
        raise ValueError("config has no num_neighbors")
    dist = _get(tree, "distance_measure", "distance_measure")
    if dist not in _DISTANCES:
        raise ValueError(f"unsupported distance_measure {dist!r} (dot product or squared L2)")
    if "brute_force" in tree:
        raise ValueError("score_brute_force is outside the MI355X tree-AH path")
    part = _get(tree, "partitioning")
    if part is None:
        raise ValueError("the MI355X path needs a partitioning (tree) stanza")
    ah = _get(tree, "hash", "asymmetric_hash")
    if ah is None:
        raise ValueError("the MI355X path needs score_ah (asymmetric hashing)")
    if _get(ah, "lookup_type") != "INT8_LUT16":
        raise ValueError("only LUT16 asymmetric hashing (hash_type='lut16') is supported")
    proj = _get(ah, "projection", default={})
    dpb = _get(proj, "num_dims_per_block")
    if dpb is None:
        dpb = _get(proj, "variable_blocks", "num_dims_per_block")
    spill = _get(part, "database_spilling")
    reorder = _get(tree, "exact_reordering", "approx_num_neighbors")
    if _get(tree, "exact_reordering", "fixed_point", "enabled") or \
            _get(tree, "exact_reordering", "bfloat16", "enabled"):
        raise ValueError("quantized reordering is not supported (float32 reorder only)")
    return SearchConfig(
        num_neighbors=int(nn), metric=_DISTANCES[dist],
        num_leaves=int(_get(part, "num_children")),
        leaves_to_search=int(_get(part, "query_spilling", "max_spill_centers")),
        training_iterations=int(_get(part, "max_clustering_iterations", default=12)),
        training_sample_size=int(_get(part, "expected_sample_size", default=100000)),
        dims_per_block=int(dpb or 2),
        residual=bool(_get(ah, "use_residual_quantization", default=False)),
        ah_training_iterations=int(_get(ah, "max_clustering_iterations", default=10)),
        ah_training_sample_size=int(_get(ah, "expected_sample_size", default=100000)),
        reorder_num_neighbors=None if reorder is None else int(reorder),
        soar_lambda=None if spill is None else float(_get(spill, "orthogonality_amplification_lambda", default=1.5)),
        overretrieve_factor=float(_get(spill, "overretrieve_factor", default=2.0)) if spill else 2.0,
        noise_shaping_threshold=_noise_shaping(ah),
        raw=tree)
