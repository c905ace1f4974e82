"""The search's alternative device paths against the oracle and each other.

These switches select kernels without changing any result (all are read
when a handle is created):

  * SMX_NARROW -- 16-slot scan tiles (v_smfmac_i32_16x16x128_i8): 0 none
    (32-slot tiles only), 1 by density (16-slot tiles only below 32 queries
    per leaf on average), 2 16-slot tiles only;
  * SMX_FUSED_WORKLIST=0 / SMX_SERIAL_WORKLIST=0 -- the work list from its
    three launches (as above 4096 leaves), on the seed's stream or on the
    side stream;
  * SMX_DENSE_FIRST=0 -- the all-sparse 32-slot tile at K % 4 == 2 instead
    of the dense-first one;
  * chunk_tiles (smx_set_tuning) -- tiles per work item, down to the
    smallest accepted (8): the most work items per call, the case the item
    buffer (MaxItems) is sized for, in every tile mode.

Every combination must give the oracle's ids and distance bits
(tree_ah_hybrid_residual.cc:631-846), and every tile mode ranks the same
seed values, so the candidates that pass the thresholds -- mean_candidates
-- are identical across the paths.
"""
import os

import numpy as np
import pytest

from tests.conftest import make_index

pytestmark = pytest.mark.gpu

PATHS = [({"SMX_NARROW": n}, 0) for n in "012"] + [
    # the smallest work items: the item buffer's worst case, 16-slot only
    ({"SMX_NARROW": "2"}, 8), ({"SMX_NARROW": "1"}, 8), ({"SMX_NARROW": "0"}, 16),
    # the work list by its three launches: before the seed on one stream, and
    # on the side stream beside it (the paths above 4096 leaves)
    ({"SMX_NARROW": "1", "SMX_FUSED_WORKLIST": "0"}, 0),
    ({"SMX_NARROW": "2", "SMX_FUSED_WORKLIST": "0", "SMX_SERIAL_WORKLIST": "0"}, 8),
    # the all-sparse 32-slot tile where the dense-first one would run
    ({"SMX_NARROW": "0", "SMX_DENSE_FIRST": "0"}, 0),
]


def _handle(ix, env):
    from scann_amd import _native
    old = {k: os.environ.get(k) for k in env}
    try:
        os.environ.update(env)
        return _native.NativeIndex(ix)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _search(ix, q, env, L, pre, seed, reorder=True, chunk=0):
    nat = _handle(ix, env)
    try:
        nat.set_tuning(candidates_per_query=0, seed_leaves=seed, chunk_tiles=chunk)
        nat.set_profiling(True)
        gi, gd, gc = nat.search_batched(q, L, pre, 10, reorder)
        t = nat.timings()
    finally:
        nat.close()
    return gi, gd, gc, t


def _check(oracle, ix, q, L, pre, seed, reorder=True):
    oi, od, oc = oracle.search(ix, q, L, pre, 10, reorder, oracle.MODE_IDEAL)
    cands = set()
    for env, chunk in PATHS:
        gi, gd, gc, t = _search(ix, q, env, L, pre, seed, reorder, chunk)
        tag = f"{env} chunk_tiles={chunk} L={L} pre={pre} seed={seed}"
        np.testing.assert_array_equal(gc, oc, err_msg=tag)
        np.testing.assert_array_equal(gi, oi, err_msg=tag)
        np.testing.assert_array_equal(gd.view(np.uint32), od.view(np.uint32), err_msg=tag)
        cands.add(t["mean_candidates"])
    assert len(cands) == 1, cands   # the same thresholds on every path


@pytest.fixture(scope="module")
def big_leaves():
    """Residual dot product, 100 dims (K = 26), ~4000 rows per leaf: leaves
    of many chunks, seed leaves past the seed's 4096-row budget."""
    return make_index(n=40000, d=100, leaves=10, seed=21, components=40)


@pytest.mark.parametrize("fix", ["small_dot", "small_l2"])
@pytest.mark.parametrize("seed", [1, 4])
def test_paths_match_oracle_and_each_other(oracle, fix, seed, request):
    ix, db, q = request.getfixturevalue(fix)
    _check(oracle, ix, q, 12, 100, seed)


@pytest.mark.parametrize("seed,L,pre", [(1, 3, 100), (2, 4, 200), (4, 6, 100)])
def test_paths_with_multi_chunk_leaves(oracle, big_leaves, seed, L, pre):
    ix, db, q = big_leaves
    assert np.diff(ix.leaf_offsets).max() > 3072
    _check(oracle, ix, q, L, pre, seed)


def test_paths_with_crowded_leaves(oracle, small_dot):
    """600 queries near 6 base queries: ~100 queries per visited leaf, so
    every leaf holds several query tiles (and, at chunk_tiles 8, many
    chunks)."""
    ix, db, q = small_dot
    rng = np.random.default_rng(5)
    qq = np.repeat(q[:6], 100, axis=0) + rng.normal(0, 1e-3, (600, q.shape[1])).astype(np.float32)
    qq /= np.linalg.norm(qq, axis=1, keepdims=True)
    _check(oracle, ix, qq.astype(np.float32), 12, 100, 4)


def test_paths_without_seed(oracle, small_l2):
    _check(oracle, ix=small_l2[0], q=small_l2[2], L=12, pre=100, seed=0, reorder=False)


# K = 26 scan tiles: 49, 50 and 51 AH blocks of 2 dims.  At 49 and
# 50 blocks the 32-slot tile opens with one dense i8 MFMA over its last blocks
# (at 49 with a padding block); SMX_DENSE_FIRST=0 runs the all-sparse tile;
# 51 blocks take the next K.  Each against the oracle, in both tile widths.
DENSE_FIRST_PATHS = [({"SMX_NARROW": "0", "SMX_DENSE_FIRST": df}, 0) for df in "01"] + [
    ({"SMX_NARROW": "2", "SMX_DENSE_FIRST": "1"}, 0)]


@pytest.mark.parametrize("dim", [98, 100, 102])
def test_dense_first_tiles_at_block_counts(oracle, dim):
    ix, db, q = make_index(n=5000, d=dim, leaves=24, seed=31 + dim, components=48)
    assert ix.num_blocks == dim // 2
    L, pre = 8, 100
    oi, od, oc = oracle.search(ix, q, L, pre, 10, True, oracle.MODE_IDEAL)
    for env, chunk in DENSE_FIRST_PATHS:
        gi, gd, gc, _ = _search(ix, q, env, L, pre, 4, True, chunk)
        tag = f"dim={dim} {env}"
        np.testing.assert_array_equal(gc, oc, err_msg=tag)
        np.testing.assert_array_equal(gi, oi, err_msg=tag)
        np.testing.assert_array_equal(gd.view(np.uint32), od.view(np.uint32), err_msg=tag)


def test_sub_batches_match_whole_batch(oracle, small_dot):
    """A batch above the leaf-slot budget runs as sub-batches (no
    batch-size limit, as the reference's search_batched has none).  With the
    budget lowered to 48 leaves x 20 queries, 64 queries run as 20+20+20+4
    through the host, device and shard entry points; every query's results
    equal the oracle's."""
    import torch
    ix, db, q = small_dot
    L, pre = 6, 100
    oi, od, oc = oracle.search(ix, q, L, pre, 10, True, oracle.MODE_IDEAL)
    nat = _handle(ix, {"SMX_LEAF_SLOT_BUDGET": str(ix.num_leaves * 20)})
    try:
        gi, gd, gc = nat.search_batched(q, L, pre, 10, True)
        np.testing.assert_array_equal(gc, oc)
        np.testing.assert_array_equal(gi, oi)
        np.testing.assert_array_equal(gd.view(np.uint32), od.view(np.uint32))
        dev = torch.device("cuda", 0)
        qd = torch.from_numpy(q).to(dev)
        di = torch.zeros((q.shape[0], 10), dtype=torch.int32, device=dev)
        dd = torch.zeros((q.shape[0], 10), dtype=torch.float32, device=dev)
        dc = torch.zeros(q.shape[0], dtype=torch.int32, device=dev)
        s = torch.cuda.Stream(dev)
        nat.search_batched_device(qd.data_ptr(), q.shape[0], L, pre, 10, True, di.data_ptr(),
                                  dd.data_ptr(), dc.data_ptr(), stream=s.cuda_stream)
        nat.release_stream(s.cuda_stream)   # waits for the stream's work
        np.testing.assert_array_equal(di.cpu().numpy().astype(np.uint32), oi)
        np.testing.assert_array_equal(dd.cpu().numpy().view(np.uint32), od.view(np.uint32))
        np.testing.assert_array_equal(dc.cpu().numpy(), oc)
        # one shard = the whole index: its entries then merge to the same result
        k = nat.shard_width(L, pre, 10, True)
        ent = torch.zeros((q.shape[0], k, 2), dtype=torch.int64, device=dev)
        nat.search_shard_device(qd.data_ptr(), q.shape[0], L, pre, 10, True, ent.data_ptr())
        nat.merge_shards_device(1, q.shape[0], L, pre, 10, True, ent.data_ptr(), di.data_ptr(),
                                dd.data_ptr(), dc.data_ptr())
        torch.cuda.synchronize()
        np.testing.assert_array_equal(di.cpu().numpy().astype(np.uint32), oi)
        np.testing.assert_array_equal(dd.cpu().numpy().view(np.uint32), od.view(np.uint32))
    finally:
        nat.close()
