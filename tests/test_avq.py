"""AVQ noise-shaped encoding (the builder's anisotropic_quantization_threshold):
the vectorised encoder (scann_amd.index_builder.encode_avq: numpy here, torch
on a GPU box) against the oracle's row-by-row restatement of
IndexDatapointNoiseShaped (asymmetric_hashing_impl.cc:434-503).  No reference
golden codes exist for this function: parity with the reference's own output
is unpinned; the restatement is pinned by the cited source."""
import numpy as np
import pytest

from scann_amd import index_builder, synthetic


def _data(n, d, seed):
    db = synthetic.mixture(n, d, 12, 0.9, seed=seed)
    centers = index_builder.kmeans(db, 8, 4, seed)
    lab = index_builder._assign_l2(db, centers)
    resid = db - centers[lab]
    cb = index_builder.train_codebook(resid, (d + 1) // 2, 2, 4, seed)
    return db, resid, cb


@pytest.mark.parametrize("d,threshold", [(32, 0.2), (31, 0.2), (16, 0.55)])
def test_avq_encoder_matches_oracle(oracle, d, threshold):
    db, resid, cb = _data(600, d, seed=d)
    got = index_builder.encode_avq(resid, db, cb, threshold, chunk=256)
    want = oracle.avq_encode(resid, db, cb, threshold)
    np.testing.assert_array_equal(got, want)
    # noise shaping moves some codes away from the nearest center, not all
    plain = index_builder.encode(resid, cb)
    frac = float((got != plain).mean())
    assert 0.0 < frac < 0.5


def test_avq_reduces_parallel_error(oracle):
    """The point of AVQ: the quantization error parallel to the datapoint
    shrinks (at the cost of more perpendicular error)."""
    db, resid, cb = _data(2000, 32, seed=3)
    nb = cb.shape[0]

    def parallel_err(codes):
        q = cb[np.arange(nb)[None, :], codes].reshape(len(db), -1)[:, :32]
        e = resid - q
        u = db / np.linalg.norm(db, axis=1, keepdims=True)
        return float(np.mean(np.sum(e * u, axis=1) ** 2))

    plain = index_builder.encode(resid, cb)
    avq = index_builder.encode_avq(resid, db, cb, 0.2)
    assert parallel_err(avq) < parallel_err(plain)


def test_config_routes_threshold():
    from scann_amd.config import search_config_from_text
    from scann_amd import scann_builder
    db = np.zeros((10, 8), np.float32)
    text = scann_builder.ScannBuilder(db, 5, "dot_product").tree(4, 2).score_ah(
        2, anisotropic_quantization_threshold=0.2).reorder(5).create_config()
    assert search_config_from_text(text).noise_shaping_threshold == pytest.approx(0.2)
    text = scann_builder.ScannBuilder(db, 5, "dot_product").tree(4, 2).score_ah(2).reorder(
        5).create_config()
    assert search_config_from_text(text).noise_shaping_threshold is None
