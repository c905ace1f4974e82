"""configs[3] / configs[4] at their per-rank workload density, against the oracle.

The bench's shard lines search rank 0's shard of an 8-way range split whose
leaves hold hundreds to thousands of rows each (configs[4]: ~2,500 per
rank-leaf at 125M rows / 50000 leaves).  The stand-ins of test_gpu_configs.py
hold ~2-10 rows per rank-leaf, so multi-chunk work items, the candidate-list
autocap, overflow rescans at K = 24 and the L = 2000 / pre_reorder_nn = 256
operating point that reaches recall >= 0.95 for configs[4] (bench.py sweep)
only run at this density.  Here rank 0's shard is generated and built on the
GPU as bench.py builds it (scann_amd/generate.py), then:

  * the shard as a standalone index (TreeAHIndex.standalone) on the GPU ==
    the oracle (ideal mode) on the same index, ids and distance bits, at the
    bench's operating points (tree_ah_hybrid_residual.cc:631-846);
  * the same with 512-entry candidate lists and no seed threshold, so that
    lists overflow and are rescanned on the device (the timings report the
    rescan passes);
  * the shard engine's own list -- search_shard + merge of that one list,
    the bench's N = 1 path -- == the oracle (ideal mode) on the shard itself:
    the whole index's ties (leaf << shift | leaf_row_base + row), its spill
    factor and SOAR dedupe by global id, the reorder from the members' own
    rows; global ids and distance bits, for the disjoint and the spilled
    (SOAR) shard alike.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

NQ = 64


def _shard(n, leaves, components, soar, seed, train, spread=0.9):
    from scann_amd import generate
    ds = generate.GeneratedDataset(n, 96, seed, components=components, spread=spread,
                                   device=torch.device("cuda"))
    ix = generate.build_generated_shard(
        ds, leaves, 0, 8, soar_lambda=soar, seed=seed, training_sample_size=train,
        training_iterations=4, ah_training_sample_size=100_000, ah_training_iterations=4,
        counts_from_all_ranks=False)
    return ix, ds.queries(NQ, seed + 1000)


def _check_points(oracle, ix, q, points, min_rows_per_leaf, multi_chunk_leaves):
    from scann_amd import _native
    from scann_amd.distributed import NativeShardEngine
    sizes = ix.leaf_sizes()
    assert sizes.mean() >= min_rows_per_leaf, sizes.mean()
    # leaves with more than one work-item chunk (20 tiles of 32 rows)
    assert int((sizes > 20 * 32).sum()) >= multi_chunk_leaves, int((sizes > 640).sum())
    view = ix.standalone()
    nv = _native.NativeIndex(view)
    eng = NativeShardEngine(ix)
    try:
        for lv, pre in points:
            oi, od, oc = oracle.search(view, q, lv, pre, 10, True, oracle.MODE_IDEAL, 16)
            # sized per call (autocap); then 512-entry lists without a seed
            # threshold: every scanned row is a candidate, lists overflow and
            # are rescanned on the device
            for cap, seed in ((0, 4), (512, 0)):
                nv.set_tuning(candidates_per_query=cap, seed_leaves=seed)
                nv.set_profiling(True)
                gi, gd, gc = nv.search_batched(q, lv, pre, 10, True)
                t = nv.timings()
                nv.set_profiling(False)
                np.testing.assert_array_equal(gc, oc)
                np.testing.assert_array_equal(gi, oi, err_msg=f"L={lv} pre={pre} cap={cap}")
                np.testing.assert_array_equal(gd.view(np.uint32), od.view(np.uint32))
                if cap:
                    assert t["overflow_retries"] > 0, t
            si_o, sd_o, sc_o = oracle.search(ix, q, lv, pre, 10, True, oracle.MODE_IDEAL, 16)
            if ix.disjoint:   # the view's top-k is the shard's, renumbered
                np.testing.assert_array_equal(si_o, ix.leaf_members[oi])
            qd = torch.from_numpy(q).cuda()
            k = eng.shard_width(lv, pre, 10, True)
            le = torch.empty((NQ, k, 2), dtype=torch.int64, device="cuda")
            eng.search_shard(qd, lv, pre, 10, True, le)
            si, sd, sc = eng.merge(1, le.unsqueeze(0), NQ, lv, pre, 10, True)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(sc.cpu().numpy(), sc_o)
            np.testing.assert_array_equal(si.cpu().numpy().astype(np.uint32), si_o,
                                          err_msg=f"shard engine L={lv} pre={pre}")
            np.testing.assert_array_equal(sd.cpu().numpy().view(np.uint32), sd_o.view(np.uint32))
    finally:
        nv.close()
        eng.nat.close()


def test_deep1b_shard_at_workload_density(oracle):
    """configs[4] at the bench's own density: rank 0 of 8 of the 10^9-row,
    50000-leaf dot-product index (shift 16; 125M rows, ~2,500 per
    rank-leaf), at the bench's headline L = 400 / pre = 100 and the
    recall-gate point L = 2000 / pre = 256."""
    ix, q = _shard(1_000_000_000, 50000, 1 << 17, None, 5, 1_000_000)
    assert ix.global_topn_shift == 16 and ix.disjoint
    _check_points(oracle, ix, q, [(400, 100), (2000, 256)], 2400, 1000)


def test_soar_shard_at_workload_density(oracle):
    """configs[3] at the bench's own density: rank 0 of 8 of the 10^8-row,
    10000-leaf SOAR index (shift 18, k' = 2 x pre; 12.5M rows, ~2,500
    members per rank-leaf), at the bench's L = 100 / pre = 100, the recall
    gate's L = 200 / pre = 128 and L = 1000 / pre = 256 (k' = 512 entries per
    shard list: the wide merge)."""
    ix, q = _shard(100_000_000, 10000, 512, 1.5, 4, 250_000, spread=1.6)   # bench.py's data
    assert ix.global_topn_shift == 18 and not ix.disjoint
    _check_points(oracle, ix, q, [(100, 100), (200, 128), (1000, 256)], 2400, 1000)
