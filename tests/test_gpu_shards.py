"""Range-split shards on the GPU: W shard indexes in one
process, their local lists stacked as the all-gather would deliver them, and
the merge kernel -- bit-equal to the unsharded ideal oracle and to the
unsharded GPU search, with and without SOAR spilling / reorder / per-shard
float rows."""
import numpy as np
import pytest
import torch

from scann_amd.index import TreeAHIndex
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
    big = torch.empty((1, 1, 2100, 2), dtype=torch.int64, device="cuda")
    with pytest.raises(_native.SmxError):   # k' above 2048
        nat.search_shard_device(torch.from_numpy(q[:1]).cuda().data_ptr(), 1, 12, 2100, 10, True,
                                big.data_ptr())


@pytest.mark.parametrize("world,pre", [(2, 300), (16, 300), (5, 1000)])
def test_wide_shard_lists_merge_to_the_oracle(oracle, world, pre):
    """Shard lists above 256 entries (SOAR: k' = 2 pre, tree_ah_hybrid_residual.h:
    263-267): the wide merge, in one launch (2 x 600 entries), after a partial
    round (16 x 600 > 8192 entries: groups of 13 lists) and at k' = 2000."""
    from scann_amd.distributed import NativeShardEngine
    ix, db, q = _soar_index()
    engines = [NativeShardEngine(ix.shard(r, world), device=0) for r in range(world)]
    qd = torch.from_numpy(q).cuda()
    nq = q.shape[0]
    for leaves, final, reorder in ((40, 10, True), (20, min(pre, 300), False)):
        k = engines[0].shard_width(leaves, pre, final, reorder)
        assert k == 2 * (pre if reorder else final)
        entries = torch.empty((world, nq, k, 2), dtype=torch.int64, device="cuda")
        for r, e in enumerate(engines):
            e.search_shard(qd, leaves, pre, final, reorder, entries[r])
        idx, dst, cnt = engines[0].merge(world, entries, nq, leaves, pre, final, reorder)
        torch.cuda.synchronize()
        oi, od, oc = oracle.search(ix, q, leaves, pre, final, reorder, oracle.MODE_IDEAL)
        tag = f"world={world} pre={pre} L={leaves}"
        np.testing.assert_array_equal(cnt.cpu().numpy(), oc, err_msg=tag)
        np.testing.assert_array_equal(idx.cpu().numpy().astype(np.uint32), oi, err_msg=tag)
        np.testing.assert_array_equal(dst.cpu().numpy().view(np.uint32), od.view(np.uint32),
                                      err_msg=tag)


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _two_process_rank(rank, world, port, outdir):
    """One rank of the range split in its own process: its HIP shard engine,
    the searcher's all-gather (gloo over host memory: both ranks share the one
    GPU of the test box) and the merge kernel."""
    import os
    import torch.distributed as dist
    from scann_amd.distributed import NativeShardEngine, RangeSplitSearcher
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        ix, db, q = make_index()
        eng = NativeShardEngine(ix.shard(rank, world), device=0)
        s = RangeSplitSearcher(eng, world)
        qd = torch.from_numpy(q).cuda()
        for reorder in (True, False):
            idx, dst, cnt = s.search_batched(qd, 12, 60, 10, reorder)
            torch.cuda.synchronize()
            np.savez(os.path.join(outdir, f"r{rank}_{int(reorder)}.npz"),
                     idx=idx.cpu().numpy(), dst=dst.cpu().numpy(), cnt=cnt.cpu().numpy())
        eng.nat.close()
    finally:
        dist.destroy_process_group()


def test_range_split_two_processes_match_oracle(oracle, tmp_path):
    """The HIP shard search + all-gather + merge across two processes
    (RangeSplitSearcher with NativeShardEngine, as bench.py's N-rank step runs
    it) equals the unsharded oracle on every rank."""
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(_two_process_rank, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    ix, db, q = make_index()
    for reorder in (True, False):
        oi, od, oc = oracle.search(ix, q, 12, 60, 10, reorder, oracle.MODE_IDEAL)
        for rank in range(world):
            r = np.load(tmp_path / f"r{rank}_{int(reorder)}.npz")
            np.testing.assert_array_equal(r["cnt"], oc)
            np.testing.assert_array_equal(r["idx"].astype(np.uint32), oi)
            np.testing.assert_array_equal(r["dst"].view(np.uint32), od.view(np.uint32))


def _oversized_leaf_index(spilled):
    """An index one of whose leaves exceeds the global top-N limit: 2^17 + 1
    leaves give shift 32 - 18 = 14 (at most 16384 rows per leaf), and leaf 7
    holds 20000 rows, so the whole index falls back to global-id ties
    (GlobalTopNShift = 0, tree_ah_hybrid_residual.h:234-247; the per-leaf
    path of tree_ah_hybrid_residual.cc:788-845).  With `spilled`, every row
    also sits in a second leaf (SOAR-like duplicates, dedupe by global id)."""
    rng = np.random.default_rng(77)
    nl, n, dim = (1 << 17) + 1, 40000, 16
    centers = rng.standard_normal((nl, dim)).astype(np.float32)
    centers[7] *= 3.0   # so that queries along it rank leaf 7 first
    labels = rng.integers(0, nl, n)
    labels[:20000] = 7
    members = [np.arange(n)]
    lab = [labels]
    if spilled:
        second = (labels + 1 + rng.integers(0, nl - 1, n)) % nl
        members.append(np.arange(n))
        lab.append(second)
    lab = np.concatenate(lab)
    mem = np.concatenate(members)
    order = np.lexsort((mem, lab))
    lab, mem = lab[order], mem[order].astype(np.uint32)
    offsets = np.zeros(nl + 1, np.uint64)
    offsets[1:] = np.cumsum(np.bincount(lab, minlength=nl))
    nb = dim // 2
    codebook = (0.3 * rng.standard_normal((nb, 16, 2))).astype(np.float32)
    codes = rng.integers(0, 16, (mem.shape[0], nb)).astype(np.uint8)
    db = rng.standard_normal((n, dim)).astype(np.float32)
    ix = TreeAHIndex(metric=0, dim=dim, num_blocks=nb, dims_per_block=2, residual=True,
                     centers=centers, codebook=codebook, leaf_offsets=offsets, leaf_members=mem,
                     member_codes=codes, num_datapoints=n, dataset=db)
    u = centers[7] / np.linalg.norm(centers[7])
    q = np.concatenate([10.0 * u + 0.05 * rng.standard_normal((16, dim)),
                        rng.standard_normal((16, dim))]).astype(np.float32)
    return ix, q, db


@pytest.mark.parametrize("spilled", [False, True])
@pytest.mark.parametrize("world", [4, 8])
def test_shards_without_global_topn_merge_to_the_oracle(oracle, spilled, world):
    """Range split of an index whose largest leaf exceeds 2^shift: the shards
    tie by global id and reorder from their own rows (member_rows, found by
    global id on the device); merge == unsharded GPU == ideal oracle."""
    from scann_amd import _native
    from scann_amd.distributed import NativeShardEngine
    ix, q, db = _oversized_leaf_index(spilled)
    assert ix.global_topn_shift_value() == 0 and int(ix.leaf_sizes().max()) > (1 << 14)
    whole = _native.NativeIndex(ix)
    shards = [ix.shard(r, world) for r in range(world)]
    assert all(s.member_rows is not None and s.dataset is None for s in shards)
    engines = [NativeShardEngine(s, device=0) for s in shards]
    qd = torch.from_numpy(q).cuda()
    nq = q.shape[0]
    try:
        for leaves, pre, final, reorder in ((8, 60, 10, True), (3, 40, 10, False),
                                            (50, 100, 20, True)):
            oi, od, oc = oracle.search(ix, q, leaves, pre, final, reorder, oracle.MODE_IDEAL)
            wi, wd, wc = whole.search_batched(q, leaves, pre, final, reorder)
            np.testing.assert_array_equal(wc, oc)
            np.testing.assert_array_equal(wi, oi)
            np.testing.assert_array_equal(wd.view(np.uint32), od.view(np.uint32))
            k = engines[0].shard_width(leaves, pre, final, reorder)
            ent = torch.empty((world, nq, k, 2), dtype=torch.int64, device="cuda")
            for r, e in enumerate(engines):
                e.search_shard(qd, leaves, pre, final, reorder, ent[r])
            si, sd, sc = engines[0].merge(world, ent, nq, leaves, pre, final, reorder)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(sc.cpu().numpy(), oc)
            np.testing.assert_array_equal(si.cpu().numpy().astype(np.uint32), oi)
            np.testing.assert_array_equal(sd.cpu().numpy().view(np.uint32), od.view(np.uint32))
        # a shard handle's own search_batched (k' > 256: the block select
        # finds rows by global id) == the oracle on the shard's rows under
        # their global ids
        s0 = _native.NativeIndex(shards[0])
        sh = shards[0]
        # (the oracle takes a shard's whole-index shift and spill setting)
        own = TreeAHIndex(metric=ix.metric, dim=ix.dim, num_blocks=ix.num_blocks,
                          dims_per_block=ix.dims_per_block, residual=ix.residual,
                          centers=ix.centers, codebook=ix.codebook, leaf_offsets=sh.leaf_offsets,
                          leaf_members=sh.leaf_members, member_codes=sh.member_codes,
                          num_datapoints=ix.num_datapoints, dataset=db,
                          leaf_row_base=sh.leaf_row_base, global_topn_shift=0,
                          global_spilled=spilled)
        for leaves, pre in ((20, 300), (4, 150)):
            gi, gd, gc = s0.search_batched(q, leaves, pre, 10, True)
            oi, od, oc = oracle.search(own, q, leaves, pre, 10, True, oracle.MODE_IDEAL)
            assert (gc[:16] > 0).all()
            np.testing.assert_array_equal(gc, oc)
            np.testing.assert_array_equal(gi, oi)
            np.testing.assert_array_equal(gd.view(np.uint32), od.view(np.uint32))
        s0.close()
    finally:
        whole.close()
        for e in engines:
            e.nat.close()
