"""Host-side logic of the Python mirror that needs no GPU: parameter
resolution (scann.cc:406-430), output conventions, index validation and
serialization round trips."""
import numpy as np
import pytest

from scann_amd.config import search_config_from_text
from scann_amd.index import TreeAHIndex
from scann_amd.scann_pybind import ScannNumpy

GLOVE = """num_neighbors: 10
distance_measure { distance_measure: "DotProductDistance" }
partitioning { num_children: 1000 query_spilling { spilling_type: FIXED_NUMBER_OF_CENTERS max_spill_centers: 100 } }
hash { asymmetric_hash { lookup_type: INT8_LUT16 use_residual_quantization: True
  projection { projection_type: CHUNK num_blocks: 50 num_dims_per_block: 2 } } }
exact_reordering { approx_num_neighbors: 100 fixed_point { enabled: False } }"""


def _searcher(text):
    s = ScannNumpy.__new__(ScannNumpy)
    s._cfg = search_config_from_text(text)
    return s


def test_defaults_follow_get_search_parameters():
    s = _searcher(GLOVE)
    assert s._resolve(-1, -1, -1) == (10, 100, 100)
    assert s._resolve(5, 40, 7) == (5, 40, 7)
    assert s._resolve(None, None, None) == (10, 100, 100)


def test_without_reordering_pre_equals_final():
    s = _searcher(GLOVE.replace("exact_reordering { approx_num_neighbors: 100 fixed_point { enabled: False } }", ""))
    assert s._resolve(7, 300, -1) == (7, 7, 100)


def test_quantized_reorder_rejected():
    with pytest.raises(ValueError, match="quantized reordering"):
        search_config_from_text(GLOVE.replace("enabled: False", "enabled: True"))


def test_index_validation(small_dot):
    ix = small_dot[0]
    kw = dict(metric=0, dim=ix.dim, num_blocks=ix.num_blocks, dims_per_block=2, residual=True,
              centers=ix.centers, codebook=ix.codebook, leaf_offsets=ix.leaf_offsets,
              leaf_members=ix.leaf_members, member_codes=ix.member_codes,
              num_datapoints=ix.num_datapoints)
    TreeAHIndex(**kw)
    with pytest.raises(ValueError):
        TreeAHIndex(**{**kw, "codebook": ix.codebook[:, :8]})
    bad = ix.member_codes.copy()
    bad[3, 1] = 17
    with pytest.raises(ValueError, match="4-bit"):
        TreeAHIndex(**{**kw, "member_codes": bad})
    with pytest.raises(ValueError, match="out of range"):
        TreeAHIndex(**{**kw, "num_datapoints": 5})


def test_index_save_load_roundtrip(tmp_path, small_dot, oracle):
    ix, db, q = small_dot
    ix.save(str(tmp_path))
    ix2 = TreeAHIndex.load(str(tmp_path))
    a = oracle.search(ix, q, 8, 50, 10, True)
    b = oracle.search(ix2, q, 8, 50, 10, True)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)


def test_native_import_fails_loudly_without_library(tmp_path):
    from scann_amd import _native
    with pytest.raises(ImportError, match="no CPU fallback"):
        _native.load.__wrapped__ if False else None
        old = _native._lib
        _native._lib = None
        try:
            _native.load(str(tmp_path / "missing.so"))
        finally:
            _native._lib = old
