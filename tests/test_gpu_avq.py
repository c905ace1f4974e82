"""AVQ encoding on the GPU (torch float64 path of index_builder.encode_avq)
equals the oracle's row-by-row restatement; an AVQ-built index searches
bit-exactly against the oracle like any other."""
import numpy as np
import pytest

from scann_amd import index_builder, synthetic

pytestmark = pytest.mark.gpu


def test_avq_gpu_encoder_matches_oracle(oracle):
    import torch
    assert torch.cuda.is_available()
    db = synthetic.mixture(3000, 32, 12, 0.9, seed=5)
    centers = index_builder.kmeans(db, 16, 4, 5)
    resid = db - centers[index_builder._assign_l2(db, centers)]
    cb = index_builder.train_codebook(resid, 16, 2, 4, 5)
    got = index_builder.encode_avq(resid, db, cb, 0.2, chunk=1024)
    want = oracle.avq_encode(resid, db, cb, 0.2)
    np.testing.assert_array_equal(got, want)


def test_avq_index_search_matches_oracle(oracle):
    from scann_amd import _native
    db = synthetic.mixture(8000, 32, 40, 0.9, seed=9)
    q = synthetic.mixture(48, 32, 40, 0.9, seed=109, means_seed=9)
    ix = index_builder.build_tree_ah(db, 0, 32, 2, training_iterations=4,
                                     ah_training_iterations=4, seed=9,
                                     noise_shaping_threshold=0.2)
    n = _native.NativeIndex(ix)
    gi, gd, gc = n.search_batched(q, 8, 100, 10, True)
    oi, od, oc = oracle.search(ix, q, 8, 100, 10, True, oracle.MODE_IDEAL)
    np.testing.assert_array_equal(gi, oi)
    np.testing.assert_array_equal(gd.view(np.uint32), od.view(np.uint32))
    n.close()
