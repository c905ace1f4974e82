"""The oracle's range-split shard semantics (ideal mode), on the CPU.

A shard (TreeAHIndex.shard: rows [n r / W, n (r + 1) / W) of every leaf)
keeps the whole index's tie -- leaf << shift | (leaf_row_base + local),
tree_ah_hybrid_residual.h:234-247 -- and reorders from its members' own
float rows.  The oracle honours both, so that the shard engine
(search_shard + merge, the bench's range-split path) can be checked
against it directly.  Invariants tested here:

  * the exact top-k' is shard-invariant: the W shards' pre-reorder lists,
    merged by (AH distance, whole-index tie), equal the whole index's list --
    on data with many duplicated rows, so that equal distances are common and
    only the whole-index tie decides which of them are kept;
  * a shard's reorder from member rows == the same shard with the dataset;
  * shard(0, 1) searches exactly like the whole index (ids and distance bits),
    for a disjoint and a SOAR-spilled index.
"""
import numpy as np
import pytest

from scann_amd import index_builder, synthetic


def _dup_index(metric, soar=None, seed=7):
    """An index whose rows repeat: 1500 distinct rows x 4 copies each."""
    base = synthetic.mixture(1500, 16, 12, 0.9, seed, normalize=metric == 0)
    db = np.repeat(base, 4, axis=0)
    rng = np.random.default_rng(seed)
    db = db[rng.permutation(db.shape[0])]
    ix = index_builder.build_tree_ah(db, metric, 12, 2, training_iterations=4,
                                     ah_training_iterations=4, seed=seed, soar_lambda=soar)
    q = synthetic.mixture(24, 16, 12, 0.9, seed + 100, normalize=metric == 0, means_seed=seed)
    return ix, db, q


def _whole_ties(ix):
    """global id -> whole-index tie (leaf << shift | row in the leaf)."""
    shift = ix.global_topn_shift_value()
    tie = {}
    for leaf in range(ix.num_leaves):
        b, e = int(ix.leaf_offsets[leaf]), int(ix.leaf_offsets[leaf + 1])
        for row in range(e - b):
            tie[int(ix.leaf_members[b + row])] = (leaf << shift) | row
    return tie


@pytest.mark.parametrize("world", [2, 3, 5])
def test_shard_top_k_merges_to_the_whole_index(oracle, world):
    ix, db, q = _dup_index(0)
    shift = ix.global_topn_shift_value()
    assert shift > 0 and ix.disjoint
    L, kk = 6, 60
    wi, wd, wc = oracle.search_pre_reorder(ix, q, L, kk)
    ties = _whole_ties(ix)
    lists = [oracle.search_pre_reorder(ix.shard(r, world), q, L, kk) for r in range(world)]
    for qi in range(q.shape[0]):
        ent = [(float(d[qi, j]), ties[int(i[qi, j])], int(i[qi, j]))
               for i, d, c in lists for j in range(int(c[qi]))]
        ent.sort(key=lambda t: (t[0], t[1]))
        got = [g for _, _, g in ent[:int(wc[qi])]]
        assert got == [int(x) for x in wi[qi, :wc[qi]]], qi
    # equal distances are common here: the tie decided the kept set
    assert np.mean(wd[:, 1:] == wd[:, :-1]) > 0.2


@pytest.mark.parametrize("metric,soar", [(0, None), (0, 1.5), (1, None)])
def test_shard_reorder_from_member_rows(oracle, metric, soar):
    ix, db, q = _dup_index(metric, soar)
    for r in range(3):
        own = ix.shard(r, 3, own_rows=True)
        ext = ix.shard(r, 3, own_rows=False)
        assert own.dataset is None and own.member_rows is not None
        oi, od, oc = oracle.search(own, q, 6, 40, 10, True, oracle.MODE_IDEAL, 4)
        ei, ed, ec = oracle.search(ext, q, 6, 40, 10, True, oracle.MODE_IDEAL, 4)
        np.testing.assert_array_equal(oc, ec)
        np.testing.assert_array_equal(oi, ei)
        np.testing.assert_array_equal(od.view(np.uint32), ed.view(np.uint32))
        # every result is one of the shard's members at its exact distance
        mem = set(int(x) for x in own.leaf_members)
        for qi in range(q.shape[0]):
            for j in range(int(oc[qi])):
                g = int(oi[qi, j])
                assert g in mem
                assert od[qi, j] == oracle.exact_distance(q[qi], db[g], metric)


@pytest.mark.parametrize("soar", [None, 1.5])
def test_one_shard_is_the_whole_index(oracle, soar):
    ix, db, q = _dup_index(0, soar)
    assert ix.disjoint == (soar is None)
    whole = oracle.search(ix, q, 6, 40, 10, True, oracle.MODE_IDEAL, 4)
    one = oracle.search(ix.shard(0, 1), q, 6, 40, 10, True, oracle.MODE_IDEAL, 4)
    for a, b in zip(whole, one):
        np.testing.assert_array_equal(a.view(np.uint32) if a.dtype == np.float32 else a,
                                      b.view(np.uint32) if b.dtype == np.float32 else b)
