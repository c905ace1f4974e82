"""The reference's Python API (scann_ops_pybind) end to end on the MI355X
path, mirroring the reference's own tests (scann_ops_pybind_test.py):
search vs search_batched, batched vs parallel, serialization round trip,
result shapes, and the recall of tree-AH + reorder against brute force."""
import os

import numpy as np
import pytest

from scann_amd import scann_ops_pybind, synthetic

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def data():
    db = synthetic.mixture(20000, 64, 100, 0.9, 51)
    q = synthetic.mixture(200, 64, 100, 0.9, 151, means_seed=51)
    return db, q


@pytest.fixture(scope="module")
def searcher(data):
    db, _ = data
    return scann_ops_pybind.builder(db, 10, "dot_product").tree(
        num_leaves=100, num_leaves_to_search=20, training_sample_size=20000).score_ah(
        2, anisotropic_quantization_threshold=0.2).reorder(100).build()


def test_shapes_and_dot_sign(searcher, data):
    db, q = data
    idx, dist = searcher.search_batched(q)
    assert idx.shape == (200, 10) and dist.shape == (200, 10)
    exact = -(q[:, None, :] * db[idx]).sum(-1) * -1  # dot product, larger is better
    np.testing.assert_allclose(dist, exact, rtol=1e-4, atol=1e-5)
    assert np.all(np.diff(dist, axis=1) <= 0)


def test_batched_equals_single_and_parallel(searcher, data):
    _, q = data
    bi, bd = searcher.search_batched(q[:20], leaves_to_search=30)
    pi, pd = searcher.search_batched_parallel(q[:20], leaves_to_search=30, batch_size=7)
    np.testing.assert_array_equal(bi, pi)
    np.testing.assert_array_equal(bd, pd)
    for r in range(5):
        si, sd = searcher.search(q[r], leaves_to_search=30)
        np.testing.assert_array_equal(si, bi[r])
        np.testing.assert_allclose(sd, bd[r], rtol=1e-6)


def test_recall_vs_brute_force(searcher, data):
    db, q = data
    idx, _ = searcher.search_batched(q, leaves_to_search=40)
    truth = synthetic.brute_force_topk(db, q, 10, 0)
    assert synthetic.recall_at_k(idx.astype(np.int64), truth, 10) > 0.9


def test_final_nn_override_and_padding(searcher, data):
    _, q = data
    idx, dist = searcher.search_batched(q[:3], final_num_neighbors=150, pre_reorder_num_neighbors=100)
    assert idx.shape == (3, 150)
    assert np.isnan(dist[:, 100:]).all() and (idx[:, 100:] == 0).all()


def test_serialization_roundtrip(searcher, data, tmp_path):
    _, q = data
    searcher.serialize(str(tmp_path))
    s2 = scann_ops_pybind.load_searcher(str(tmp_path))
    a = searcher.search_batched(q[:50])
    b = s2.search_batched(q[:50])
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])


def test_docids_and_squared_l2(data):
    db, q = data
    docids = [f"doc{i}" for i in range(db.shape[0])]
    s = scann_ops_pybind.builder(db, 5, "squared_l2").tree(50, 10).score_ah(2).reorder(50).build(
        docids=docids)
    idx, dist = s.search_batched(q[:4])
    assert isinstance(idx[0][0], str) and idx[0][0].startswith("doc")
    assert np.all(np.diff(dist, axis=1) >= 0)


def test_soar_searcher(data):
    db, q = data
    s = scann_ops_pybind.builder(db, 10, "dot_product").tree(
        100, 20, soar_lambda=1.5, overretrieve_factor=2.0).score_ah(2).reorder(100).build()
    idx, _ = s.search_batched(q)
    for row in idx:
        assert len(set(row.tolist())) == 10
    truth = synthetic.brute_force_topk(db, q, 10, 0)
    assert synthetic.recall_at_k(idx.astype(np.int64), truth, 10) > 0.9


def test_soar_serialization_in_reference_layout(data, tmp_path):
    """serialize -> load_searcher through the reference's artifacts layout
    (scann.cc:504-601): SOAR 2N tokenization, the soar hashed dataset and a
    relative-path assets file; results identical before and after."""
    db, q = data
    s = scann_ops_pybind.builder(db, 10, "dot_product").tree(
        100, 20, soar_lambda=1.5, overretrieve_factor=2.0).score_ah(2).reorder(100).build()
    s.serialize(str(tmp_path), relative_path=True)
    names = set(os.listdir(tmp_path))
    assert {"scann_config.pb", "scann_assets.pbtxt", "hashed_dataset_soar.npy",
            "serialized_partitioner.pb", "ah_codebook.pb", "dataset.npy"} <= names
    s2 = scann_ops_pybind.load_searcher(str(tmp_path))
    a = s.search_batched(q[:64])
    b = s2.search_batched(q[:64])
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])
    assert "INT8_LUT16" in s2.config()


def test_cpp_core_defaults_and_errors(searcher, data):
    """ScannNumpyCore (C++, scann_amd/csrc/smx_pybind.cc) resolves -1 to the
    config defaults as ScannInterface::GetSearchParametersBatched does
    (scann.cc:406-430) and maps a failed search to RuntimeError with the
    reference's prefix (scann_npy.cc:41-47)."""
    _, q = data
    core = searcher.searcher._core
    a = core.search_batched(q[:16])
    b = core.search_batched(q[:16], 10, 100, 20)
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])
    with pytest.raises(ValueError, match="two-dimensional"):
        core.search_batched(q[0])
    with pytest.raises(RuntimeError, match="Error during search: "):
        core.search_batched(q[:4, :10])   # wrong dimensionality


def test_own_format_directory_loads(searcher, data, tmp_path):
    """A directory written by TreeAHIndex.save (this package's own format)
    plus the config text loads through load_searcher / ScannNumpy as before
    and searches identically."""
    _, q = data
    d = str(tmp_path / "own")
    searcher.searcher.index.save(d)
    with open(os.path.join(d, "scann_config.pbtxt"), "w") as f:
        f.write(searcher.config())
    loaded = scann_ops_pybind.load_searcher(d)
    i0, d0 = searcher.search_batched(q)
    i1, d1 = loaded.search_batched(q)
    np.testing.assert_array_equal(i0, i1)
    np.testing.assert_array_equal(d0, d1)
