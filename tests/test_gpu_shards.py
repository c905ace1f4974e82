"""Range-split shards on the GPU: W shard indexes in one
process, their local lists stacked as the all-gather would deliver them, and
the merge kernel -- bit-equal to the unsharded ideal oracle and to the
unsharded GPU search, with and without SOAR spilling / reorder / per-shard
float rows."""
import numpy as np
import pytest
import torch

from tests.conftest import make_index

pytestmark = pytest.mark.gpu


def _soar_index():
    from scann_amd import index_builder, synthetic
    db = synthetic.mixture(6000, 32, 48, 0.9, 41)
    q = synthetic.mixture(48, 32, 48, 0.9, 141, means_seed=41)
    ix = index_builder.build_tree_ah(db, 0, 40, 2, training_iterations=4,
                                     ah_training_iterations=4, soar_lambda=1.5, seed=41)
    return ix, db, q


@pytest.mark.parametrize("world", [1, 2, 3])
@pytest.mark.parametrize("kind", ["dot", "soar", "dot_dataset_rows"])
def test_shard_merge_equals_unsharded(oracle, world, kind):
    from scann_amd import _native
    from scann_amd.distributed import NativeShardEngine, RangeSplitSearcher
    ix, db, q = _soar_index() if kind == "soar" else make_index()
    own = kind != "dot_dataset_rows"
    engines = [NativeShardEngine(ix.shard(r, world, own_rows=own), device=0) for r in range(world)]
    whole = _native.NativeIndex(ix)
    qd = torch.from_numpy(q).cuda()
    nq = q.shape[0]
    for leaves, pre, final, reorder in ((12, 60, 10, True), (6, 40, 10, False), (40, 100, 20, True)):
        k = engines[0].shard_width(leaves, pre, final, reorder)
        entries = torch.empty((world, nq, k, 2), dtype=torch.int64, device="cuda")
        for r, e in enumerate(engines):
            e.search_shard(qd, leaves, pre, final, reorder, entries[r])
        idx, dst, cnt = engines[0].merge(world, entries, nq, leaves, pre, final, reorder)
        torch.cuda.synchronize()
        gi = idx.cpu().numpy().astype(np.uint32)
        gd = dst.cpu().numpy()
        oi, od, oc = oracle.search(ix, q, leaves, pre, final, reorder, oracle.MODE_IDEAL)
        np.testing.assert_array_equal(cnt.cpu().numpy(), oc)
        np.testing.assert_array_equal(gi, oi)
        np.testing.assert_array_equal(gd.view(np.uint32), od.view(np.uint32))
        wi, wd, wc = whole.search_batched(q, leaves, pre, final, reorder)
        np.testing.assert_array_equal(gi, wi)
        if world == 1:   # the searcher's own path (no process group needed)
            s = RangeSplitSearcher(engines[0], world=1)
            i2, d2, c2 = s.search_batched(qd, leaves, pre, final, reorder)
            np.testing.assert_array_equal(i2.cpu().numpy().astype(np.uint32), oi)


def test_shard_errors(oracle):
    from scann_amd import _native
    ix, db, q = make_index()
    s = ix.shard(0, 2)
    nat = _native.NativeIndex(s)
    with pytest.raises(_native.SmxError):
        nat.shard_width(12, 0, 10, True)   # pre_nn must be > 0 with reorder
    big = torch.empty((1, 1, 300, 2), dtype=torch.int64, device="cuda")
    with pytest.raises(_native.SmxError):
        nat.search_shard_device(torch.from_numpy(q[:1]).cuda().data_ptr(), 1, 12, 300, 10, True,
                                big.data_ptr())
