"""Multi-process (gloo, world_size 2) coverage of the multi-GPU paths.

The range-split orchestration (``scann_amd.distributed.RangeSplitSearcher``:
local lists -> the one all-gather -> merge) runs here on CPU with a test
engine whose per-shard lists come from the unsharded CPU oracle restricted to
the shard's rows, and whose merge is a numpy mirror of merge_shards_kernel.
The result must equal the unsharded oracle search, which pins the sharding
invariants the HIP shard/merge kernels rely on (row slices, whole-index ties,
shard-invariance of the exact top-k').  The HIP kernels themselves are checked
in tests/test_gpu_shards.py.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from scann_amd import distributed as sd
from tests.conftest import make_index


def _ordered(d):
    u = (np.asarray(d, np.float32) + np.float32(0.0)).view(np.uint32).astype(np.uint64)
    return np.where(u & 0x80000000, (~u) & 0xFFFFFFFF, u | 0x80000000)


class OracleShardEngine:
    """Test engine: shard lists from the unsharded oracle (CPU tensors)."""

    def __init__(self, ix, db, rank, world, oracle):
        self.ix, self.db, self.oracle = ix, db, oracle
        self.shard = ix.shard(rank, world)
        self.shift = ix.global_topn_shift_value()
        sizes = ix.leaf_sizes()
        self.lo = self.shard.leaf_row_base.astype(np.int64)
        self.hi = self.lo + self.shard.leaf_sizes()
        # global id -> (leaf, row within the whole leaf); disjoint index
        self.leaf_of = np.repeat(np.arange(ix.num_leaves), sizes)
        self.row_of = np.concatenate([np.arange(n) for n in sizes])
        self.pos = np.empty(ix.num_datapoints, np.int64)
        self.pos[ix.leaf_members] = np.arange(ix.num_members)

    def shard_width(self, leaves, pre_nn, final_nn, reorder):
        return pre_nn if reorder else final_nn

    def search_shard(self, queries, leaves, pre_nn, final_nn, reorder, out):
        q = queries.numpy()
        k = out.shape[1]
        ids, d, cnt = self.oracle.search_pre_reorder(self.ix, q, leaves, self.ix.num_members,
                                                     self.oracle.MODE_IDEAL)
        words = np.zeros((q.shape[0], k, 2), np.uint64)
        words[:, :, 0] = np.uint64(0xFFFFFFFFFFFFFFFF)
        for i in range(q.shape[0]):
            gi, gd = ids[i, :cnt[i]], d[i, :cnt[i]]
            p = self.pos[gi]
            leaf, row = self.leaf_of[p], self.row_of[p]
            mine = (row >= self.lo[leaf]) & (row < self.hi[leaf])
            gi, gd, leaf, row = gi[mine][:k], gd[mine][:k], leaf[mine][:k], row[mine][:k]
            tie = ((leaf.astype(np.uint64) << np.uint64(self.shift)) | row.astype(np.uint64)
                   if self.shift > 0 else gi.astype(np.uint64))
            ex = (np.array([self.oracle.exact_distance(q[i], self.db[g], self.ix.metric) for g in gi],
                           np.float32) if reorder else gd)
            words[i, :len(gi), 0] = (_ordered(gd) << np.uint64(32)) | tie
            words[i, :len(gi), 1] = gi.astype(np.uint64) | (ex.astype(np.float32).view(np.uint32)
                                                            .astype(np.uint64) << np.uint64(32))
        out.copy_(torch.from_numpy(words.view(np.int64)))

    def merge(self, world, entries, nq, leaves, pre_nn, final_nn, reorder):
        e = entries.numpy().view(np.uint64)
        idx = np.zeros((nq, final_nn), np.uint32)
        dst = np.full((nq, final_nn), np.nan, np.float32)
        cnt = np.zeros(nq, np.int32)
        for i in range(nq):
            keys = e[:, i, :, 0].ravel()
            w1 = e[:, i, :, 1].ravel()
            ok = keys != np.uint64(0xFFFFFFFFFFFFFFFF)
            keys, w1 = keys[ok], w1[ok]
            order = np.argsort(keys, kind="stable")[: (pre_nn if reorder else final_nn)]
            gid = (w1[order] & np.uint64(0xFFFFFFFF)).astype(np.uint32)
            ex = (w1[order] >> np.uint64(32)).astype(np.uint32).view(np.float32)
            approx = ((keys[order] >> np.uint64(32)).astype(np.uint32))
            dvals = ex if reorder else np.where(approx & 0x80000000, approx & 0x7FFFFFFF,
                                                ~approx).astype(np.uint32).view(np.float32)
            fin = np.lexsort((gid, _ordered(dvals)))[:final_nn]
            m = len(fin)
            idx[i, :m], dst[i, :m], cnt[i] = gid[fin], dvals[fin], m
        return idx, dst, cnt


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, outdir):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        from oracle import binding as oracle
        ix, db, q = make_index()
        searcher = sd.RangeSplitSearcher(OracleShardEngine(ix, db, rank, world, oracle), world)
        for reorder in (True, False):
            idx, dst, cnt = searcher.search_batched(torch.from_numpy(q[:24]), 12, 60, 10, reorder)
            np.savez(os.path.join(outdir, f"r{rank}_{int(reorder)}.npz"), idx=idx, dst=dst, cnt=cnt)
        # replica slices cover the batch exactly once
        b, e = sd.query_slice(q.shape[0], rank, world)
        t = torch.tensor([e - b], dtype=torch.int64)
        dist.all_reduce(t)
        np.save(os.path.join(outdir, f"slices{rank}.npy"), t.numpy())
    finally:
        dist.destroy_process_group()


def test_range_split_gloo_world2_matches_unsharded_oracle(oracle, tmp_path):
    world = 2
    mp.spawn(_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    ix, db, q = make_index()
    for reorder in (True, False):
        oi, od, oc = oracle.search(ix, q[:24], 12, 60, 10, reorder, oracle.MODE_IDEAL)
        for rank in range(world):
            r = np.load(tmp_path / f"r{rank}_{int(reorder)}.npz")
            np.testing.assert_array_equal(r["cnt"], oc)
            np.testing.assert_array_equal(r["idx"], oi)
            np.testing.assert_array_equal(r["dst"].view(np.uint32), od.view(np.uint32))
    for rank in range(world):
        assert int(np.load(tmp_path / f"slices{rank}.npy")[0]) == q.shape[0]


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_rows_partition_every_leaf(world):
    ix, db, q = make_index()
    shards = [ix.shard(r, world) for r in range(world)]
    shift = ix.global_topn_shift_value()
    assert shift > 0
    for l in range(ix.num_leaves):
        b, e = int(ix.leaf_offsets[l]), int(ix.leaf_offsets[l + 1])
        got = []
        for s in shards:
            sb, se = int(s.leaf_offsets[l]), int(s.leaf_offsets[l + 1])
            base = int(s.leaf_row_base[l])
            np.testing.assert_array_equal(s.leaf_members[sb:se], ix.leaf_members[b + base:b + base + se - sb])
            np.testing.assert_array_equal(s.member_codes[sb:se], ix.member_codes[b + base:b + base + se - sb])
            got.append((base, se - sb))
        # contiguous, ordered, complete
        pos = 0
        for base, n in got:
            assert base == pos
            pos += n
        assert pos == e - b
    for s in shards:
        assert s.global_topn_shift == shift and s.disjoint
        assert s.dataset is None and s.member_rows.shape == (s.num_members, ix.dim)
        np.testing.assert_array_equal(s.member_rows, db[s.leaf_members])


def test_query_slices_cover_batch():
    for nq in (0, 1, 7, 1000):
        for world in (1, 2, 3, 8):
            spans = [sd.query_slice(nq, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == nq
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))


def _split_rank_main(rank, world, port, outdir):
    """Strong scaling on CPU: one 61-query batch split over `world` gloo
    ranks (uneven slices), each slice searched by the oracle, the slices
    all-gathered by SplitBatchSearcher."""
    import torch.distributed as dist
    from scann_amd import distributed as sd
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        from oracle import binding as oracle
        ix, db, q = make_index()

        def search(qs):
            i, d, c = oracle.search(ix, qs.numpy(), 12, 60, 10, True, oracle.MODE_IDEAL)
            return (torch.from_numpy(i.astype(np.int64)), torch.from_numpy(d),
                    torch.from_numpy(c.astype(np.int32)))

        s = sd.SplitBatchSearcher(search, rank, world)
        idx, dst, cnt = s.search_batched(torch.from_numpy(q[:61]))
        np.savez(os.path.join(outdir, f"split{rank}.npz"), idx=idx.numpy(), dst=dst.numpy(),
                 cnt=cnt.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_split_batch_gloo_concatenates_to_the_one_rank_result(oracle, tmp_path, world):
    """bench.py --scaling strong's split (scann.cc:478-501 chunking across
    ranks): every rank ends with the 1-rank result of the whole batch, bit for
    bit."""
    mp.spawn(_split_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    ix, db, q = make_index()
    oi, od, oc = oracle.search(ix, q[:61], 12, 60, 10, True, oracle.MODE_IDEAL)
    for rank in range(world):
        r = np.load(tmp_path / f"split{rank}.npz")
        np.testing.assert_array_equal(r["idx"], oi.astype(np.int64))
        np.testing.assert_array_equal(r["dst"].view(np.uint32), od.view(np.uint32))
        np.testing.assert_array_equal(r["cnt"], oc)
