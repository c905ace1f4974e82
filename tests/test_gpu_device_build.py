"""The device index build (scann_amd/device_builder.py over the HIP kernels of
smx_builder.hip / smx_sort.hip) against restatements:

* smx_avq_encode == the oracle's orc_avq_encode (IndexDatapointNoiseShaped,
  asymmetric_hashing_impl.cc:434-503) byte for byte, odd dims (zero-padded
  last block), dims_per_block 2 and 3, several thresholds;
* smx_block_encode == a float32 numpy restatement of the nearest codebook
  center per block (squared L2 in coordinate order, first minimum);
* the fixed-point k-means mean step: equal to float64 means within float32
  rounding, and the same bits on every run (order-independent sums);
* smx_group_by_leaf == numpy's lexsort of (leaf, id), offsets == cumsum;
* an index built entirely on the device searches bit-exactly like the oracle
  on that index, with SOAR and with AVQ codes.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.mark.parametrize("n,dim,dpb,thr", [(700, 17, 2, 0.2), (500, 32, 2, 0.5),
                                           (300, 100, 2, 0.3), (400, 31, 3, 0.2),
                                           (64, 96, 2, 1.0)])
def test_avq_kernel_matches_oracle(oracle, n, dim, dpb, thr):
    from scann_amd import device_builder as db
    rng = np.random.default_rng(dim * 7 + n)
    nb = -(-dim // dpb)
    x = rng.standard_normal((n, dim)).astype(np.float32)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    c = rng.standard_normal((8, dim)).astype(np.float32) * 0.3
    r = (x - c[rng.integers(0, 8, n)]).astype(np.float32)
    cb = (rng.standard_normal((nb, 16, dpb)) * 0.2).astype(np.float32)
    got = db.avq_encode(_dev(r), _dev(x), _dev(cb), thr).cpu().numpy()
    want = oracle.avq_encode(r, x, cb, thr)
    np.testing.assert_array_equal(got, want)
    plain = db.block_encode(_dev(r), _dev(cb)).cpu().numpy()
    # unit rows: eta = t^2 / ((1 - t^2) / (dim - 1)); at t >= 1 the parallel
    # cost multiplier is infinite or negative (still bit-equal above)
    if thr < 1.0 and (thr * thr) / ((1.0 - thr * thr) / (dim - 1.0)) > 1.0:
        assert (got != plain).any()     # noise shaping moved some codes


def _block_encode_ref(r, cb):
    n, dim = r.shape
    nb, _, dpb = cb.shape
    pad = np.zeros((n, nb * dpb), np.float32)
    pad[:, :dim] = r
    v = pad.reshape(n, nb, 1, dpb) - cb[None]          # float32
    d = np.zeros((n, nb, 16), np.float32)
    for i in range(dpb):
        d = (d + v[..., i] * v[..., i]).astype(np.float32)
    return d.argmin(-1).astype(np.uint8)


@pytest.mark.parametrize("n,dim,dpb", [(3000, 100, 2), (1000, 33, 2), (500, 96, 4)])
def test_block_encode_matches_restatement(n, dim, dpb):
    from scann_amd import device_builder as db
    rng = np.random.default_rng(n + dim)
    nb = -(-dim // dpb)
    r = rng.standard_normal((n, dim)).astype(np.float32)
    cb = rng.standard_normal((nb, 16, dpb)).astype(np.float32)
    got = db.block_encode(_dev(r), _dev(cb)).cpu().numpy()
    np.testing.assert_array_equal(got, _block_encode_ref(r, cb))


def test_kmeans_mean_step_exact_and_deterministic():
    from scann_amd import _native
    from scann_amd import device_builder as db
    rng = np.random.default_rng(5)
    n, d, k = 20000, 24, 37
    x = rng.standard_normal((n, d)).astype(np.float32) * 3.0
    lab = rng.integers(0, k - 1, n).astype(np.int32)     # center k-1 stays empty
    xd, ld = _dev(x), _dev(lab)
    scale = db.fixed_point_scale(float(np.abs(x).max()), n)
    outs = []
    for _ in range(2):
        sums = torch.zeros(k * d, dtype=torch.int64, device="cuda")
        cnt = torch.zeros(k, dtype=torch.int32, device="cuda")
        cen = torch.full((k, d), 7.0, dtype=torch.float32, device="cuda")
        lib = _native.load()
        _native.check(lib.smx_kmeans_accumulate(db._p(xd), n, d, db._p(ld), k, scale, db._p(sums),
                                                db._p(cnt), None), "acc")
        _native.check(lib.smx_kmeans_finalize(db._p(sums), db._p(cnt), k, d, scale, db._p(cen),
                                              None), "fin")
        torch.cuda.synchronize()
        outs.append(cen.cpu().numpy())
    np.testing.assert_array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32))
    want = np.zeros((k, d))
    np.add.at(want, lab, x.astype(np.float64))
    counts = np.bincount(lab, minlength=k)
    want[:k - 1] /= counts[:k - 1, None]
    np.testing.assert_allclose(outs[0][:k - 1], want[:k - 1], rtol=2e-6, atol=1e-6)
    assert np.all(outs[0][k - 1] == 7.0)                 # empty center untouched


@pytest.mark.parametrize("m,k", [(100000, 1000), (5000, 50000), (1, 3), (0, 4)])
def test_group_by_leaf_matches_lexsort(m, k):
    from scann_amd import device_builder as db
    rng = np.random.default_rng(m + k)
    lab = rng.integers(0, k, m).astype(np.int32)
    ids = rng.permutation(max(m, 1))[:m].astype(np.int32)
    off, mem, ml = db.group_by_leaf(_dev(lab) if m else torch.zeros(0, dtype=torch.int32,
                                                                     device="cuda"),
                                    _dev(ids) if m else torch.zeros(0, dtype=torch.int32,
                                                                    device="cuda"), k)
    order = np.lexsort((ids, lab))
    np.testing.assert_array_equal(mem.cpu().numpy(), ids[order])
    np.testing.assert_array_equal(ml.cpu().numpy(), lab[order])
    want = np.zeros(k + 1, np.int64)
    want[1:] = np.cumsum(np.bincount(lab, minlength=k))
    np.testing.assert_array_equal(off.cpu().numpy(), want)


@pytest.mark.parametrize("soar,avq", [(False, False), (True, False), (False, True)])
def test_device_built_index_search_parity(oracle, soar, avq):
    from scann_amd import _native, synthetic
    from scann_amd import device_builder as db
    x = synthetic.mixture(20000, 64, 64, 0.9, seed=11)
    q = synthetic.mixture(48, 64, 64, 0.9, seed=111, means_seed=11)
    tm = {}
    ix = db.build_tree_ah(x, 0, 64, 2, training_iterations=6, ah_training_iterations=6, seed=3,
                          soar_lambda=1.5 if soar else None,
                          noise_shaping_threshold=0.2 if avq else None, timings=tm)
    assert set(tm) >= {"partitioner", "tokenize", "group", "codebook", "encode", "total"}
    assert ix.num_members == (2 if soar else 1) * 20000
    off = ix.leaf_offsets
    for leaf in range(64):   # members ascending within a leaf
        mm = ix.leaf_members[off[leaf]:off[leaf + 1]]
        assert np.all(np.diff(mm.astype(np.int64)) > 0)
    nat = _native.NativeIndex(ix)
    gi, gd, gc = nat.search_batched(q, 8, 100, 10, True)
    oi, od, oc = oracle.search(ix, q, 8, 100, 10, True, oracle.MODE_IDEAL)
    nat.close()
    np.testing.assert_array_equal(gi, oi)
    np.testing.assert_array_equal(gd.view(np.uint32), od.view(np.uint32))
    truth = synthetic.brute_force_topk(x, q, 10, 0)
    assert synthetic.recall_at_k(gi.astype(np.int64), truth, 10) > 0.8


@pytest.mark.parametrize("dim,dpb", [(100, 2), (900, 2)])
def test_codebook_accumulate_sums(dim, dpb):
    """Every block's 16-center sums and counts at once, LDS-privatised (100
    dims) or straight to global memory (900 dims: 450 blocks); the means equal
    float64 means."""
    from scann_amd import _native
    from scann_amd import device_builder as db
    rng = np.random.default_rng(dim)
    n, nb = 3000, -(-dim // dpb)
    r = rng.standard_normal((n, dim)).astype(np.float32)
    codes = rng.integers(0, 16, (n, nb)).astype(np.uint8)
    scale = db.fixed_point_scale(float(np.abs(r).max()), n)
    sums = torch.zeros(nb * 16 * dpb, dtype=torch.int64, device="cuda")
    cnt = torch.zeros(nb * 16, dtype=torch.int32, device="cuda")
    cen = torch.zeros((nb * 16, dpb), dtype=torch.float32, device="cuda")
    rd, cd = _dev(r), _dev(codes)
    lib = _native.load()
    _native.check(lib.smx_codebook_accumulate(db._p(rd), n, dim, db._p(cd), nb, dpb, scale,
                                              db._p(sums), db._p(cnt), None), "acc")
    _native.check(lib.smx_kmeans_finalize(db._p(sums), db._p(cnt), nb * 16, dpb, scale,
                                          db._p(cen), None), "fin")
    torch.cuda.synchronize()
    pad = np.zeros((n, nb * dpb))
    pad[:, :dim] = r
    want = np.zeros((nb, 16, dpb))
    wc = np.zeros((nb, 16), np.int64)
    for b in range(nb):
        np.add.at(want[b], codes[:, b], pad[:, b * dpb:(b + 1) * dpb])
        wc[b] = np.bincount(codes[:, b], minlength=16)
    np.testing.assert_array_equal(cnt.cpu().numpy().reshape(nb, 16), wc)
    np.testing.assert_allclose(cen.cpu().numpy().reshape(nb, 16, dpb),
                               want / np.maximum(wc, 1)[..., None], rtol=2e-6, atol=1e-6)
