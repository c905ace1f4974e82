"""GPU parity for indexes with more leaves than one LDS-resident selection holds.

Deep1B's configuration (BASELINE.json configs[4]) has 50000 leaves: the
per-query top-L over 50000 partition scores (KMeansTreePartitioner::
TokensForDatapointWithSpillingBatched, kmeans_tree_partitioner.cc:643-730) is
selected from global memory (topl_select_global_kernel) and the query-by-leaf
inversion (InvertCentersToSearch, tree_ah_hybrid_residual.cc:610-622) counts
in LDS leaf ranges.  The indexes here are synthetic but valid: random centers
(with exact duplicates, so partition scores tie and the (distance, leaf index)
order decides), random leaf assignment (many empty leaves), a random codebook
and codes -- the parity bar is the oracle on the same index, bit for bit.
"""
import numpy as np
import pytest

from scann_amd.index import TreeAHIndex

pytestmark = pytest.mark.gpu


def _random_index(nl, n, dim, metric, seed, dup=True, nq=24):
    rng = np.random.default_rng(seed)
    centers = rng.standard_normal((nl, dim)).astype(np.float32)
    if dup:   # every center of the second half repeats one of the first half
        h = nl // 2
        centers[h:2 * h] = centers[rng.permutation(h)]
    labels = np.sort(rng.integers(0, nl, n))
    ids = np.arange(n, dtype=np.uint32)
    counts = np.bincount(labels, minlength=nl)
    offsets = np.zeros(nl + 1, np.uint64)
    offsets[1:] = np.cumsum(counts)
    nb = dim // 2
    codebook = (0.3 * rng.standard_normal((nb, 16, 2))).astype(np.float32)
    codes = rng.integers(0, 16, (n, nb)).astype(np.uint8)
    db = rng.standard_normal((n, dim)).astype(np.float32)
    ix = TreeAHIndex(metric=metric, dim=dim, num_blocks=nb, dims_per_block=2,
                     residual=metric == 0, centers=centers, codebook=codebook,
                     leaf_offsets=offsets, leaf_members=ids, member_codes=codes,
                     num_datapoints=n, dataset=db)
    q = rng.standard_normal((nq, dim)).astype(np.float32)
    return ix, q


@pytest.fixture(scope="module")
def native():
    from scann_amd import _native
    return _native


@pytest.mark.parametrize("nl,metric,dim", [(20000, 0, 96), (50000, 1, 100), (5000, 1, 128)])
def test_partition_scores_several_center_tiles_per_block(native, oracle, nl, metric, dim):
    """Above 1024 64x64 tiles a partition block takes several consecutive
    center tiles (its query tile staged once, the next center tile's loads in
    flight; smx_kernels.hip partition_scores_kernel): 200 queries = 4 query
    tiles, so 20000 / 50000 leaves give 2 / 4 center tiles per block (the last
    block a partial run), 5000 leaves one (control).  Both metrics, dims with
    and without 16-dim padding."""
    ix, q = _random_index(nl, 2 * nl, dim, metric, seed=3 * nl + metric, nq=200)
    n = native.NativeIndex(ix)
    for L in (10, 100):
        gl, gd = n.partition_topl(q, L)
        ol, od = oracle.partition_topl(q, ix.centers, ix.metric, L)
        np.testing.assert_array_equal(gl, ol)
        np.testing.assert_array_equal(gd.view(np.uint32), od.view(np.uint32))


@pytest.mark.parametrize("nl,metric", [(1000, 0), (2048, 1), (5000, 0), (10000, 1), (20000, 0),
                                       (20000, 1), (50000, 0)])
def test_partition_topl_many_leaves(native, oracle, nl, metric):
    ix, q = _random_index(nl, 2 * nl, 16, metric, seed=nl + metric)
    n = native.NativeIndex(ix)
    for L in (1, 2, 99, 100, 1000, 4096):
        gl, gd = n.partition_topl(q, L)
        ol, od = oracle.partition_topl(q, ix.centers, ix.metric, L)
        np.testing.assert_array_equal(gl, ol)
        np.testing.assert_array_equal(gd.view(np.uint32), od.view(np.uint32))


@pytest.mark.parametrize("nl", [1000, 5000, 20000, 50000])
def test_partition_topl_all_ties(native, oracle, nl):
    """Every center identical: the L lowest leaf indices, in index order
    (wave select, block select, global-memory select, and the sampled
    threshold's fallback: every key ties the sampled threshold)."""
    ix, q = _random_index(nl, 30000, 16, 0, seed=5, dup=False)
    ix.centers[:] = ix.centers[0]
    n = native.NativeIndex(ix)
    for L in (1, 37, 300, 700, 4096):
        gl, gd = n.partition_topl(q, L)
        ol, od = oracle.partition_topl(q, ix.centers, ix.metric, L)
        np.testing.assert_array_equal(gl, ol)
        np.testing.assert_array_equal(gl[0][:min(L, nl)], np.arange(min(L, nl)))
        np.testing.assert_array_equal(gd.view(np.uint32), od.view(np.uint32))


@pytest.mark.parametrize("nl,metric", [(10000, 0), (20000, 0), (50000, 0), (20000, 1), (70000, 0)])
def test_search_many_leaves_matches_oracle(native, oracle, nl, metric):
    """(70000 leaves: past 65536, the work list's block sums take two
    rounds and the global top-N shift drops to 15.)"""
    ix, q = _random_index(nl, 2 * nl, 16, metric, seed=7 * nl + metric)
    n = native.NativeIndex(ix)
    for leaves, pre in ((50, 100), (400, 100)):
        gi, gd, gc = n.search_pre_reorder(q, leaves, pre)
        oi, od, oc = oracle.search_pre_reorder(ix, q, leaves, pre, oracle.MODE_IDEAL)
        np.testing.assert_array_equal(gc, oc)
        np.testing.assert_array_equal(gi, oi)
        np.testing.assert_array_equal(gd.view(np.uint32), od.view(np.uint32))
        gi, gd, gc = n.search_batched(q, leaves, pre, 10, True)
        oi, od, oc = oracle.search(ix, q, leaves, pre, 10, True, oracle.MODE_IDEAL)
        np.testing.assert_array_equal(gi, oi)
        np.testing.assert_array_equal(gd.view(np.uint32), od.view(np.uint32))


@pytest.mark.parametrize("ntie", [100, 600, 3000])
def test_partition_topl_crowded_ties(native, oracle, ntie):
    """50000 leaves of which `ntie` share one center next to every query: the
    L nearest are (mostly) one tie group, ordered by leaf index -- the sampled
    kernel's crowded-bin and in-place sort paths."""
    ix, q = _random_index(50000, 60000, 16, 0, seed=11 + ntie, dup=False)
    rng = np.random.default_rng(ntie)
    tied = rng.choice(50000, ntie, replace=False)
    ix.centers[tied] = ix.centers[tied[0]]
    q[:] = ix.centers[tied[0]] + 0.01 * rng.standard_normal(q.shape).astype(np.float32)
    n = native.NativeIndex(ix)
    for L in (50, 400, 2000):
        gl, gd = n.partition_topl(q, L)
        ol, od = oracle.partition_topl(q, ix.centers, ix.metric, L)
        np.testing.assert_array_equal(gl, ol)
        np.testing.assert_array_equal(gd.view(np.uint32), od.view(np.uint32))
