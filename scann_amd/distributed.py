"""Multi-GPU search: one process per GPU over ``torch.distributed``.

Replicas (configs whose index fits one GPU, e.g. glove): every rank holds the
whole index.  Weak scaling (``bench.py --gpus N``, the default): each rank
serves its own query batches, no collective.  Strong scaling
(``SplitBatchSearcher``, ``bench.py --scaling strong``): ONE batch is split
over the ranks by ``query_slice`` -- the chunking of the reference's
SearchBatchedParallel (scann/scann_ops/cc/scann.cc:478-501), across GPUs
instead of threads -- and the slices' results are all-gathered, so every rank
holds the whole batch's results in query order.

Range split (configs whose floats or codes do not fit one GPU): rank r holds
rows [n*r/W, n*(r+1)/W) of *every* leaf (``TreeAHIndex.shard``), which stays
balanced whatever the query popularity.  Per batch each rank computes its
exact local top-k' by (approximate distance, whole-index tie) together with
the exact distances of its own rows (``smx_search_shard_device``); ONE
all-gather of the [nq][k'] 16-byte entries (RCCL over xGMI for backend
"nccl"); then every rank runs the merge kernel (``smx_merge_shards_device``):
the exact top-k' under a total order is shard-invariant, so the result equals
the unsharded search bit for bit.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.distributed as dist

ENTRY_INT64S = 2   # smx_shard_entry {u64 key; u32 id; f32 exact} as two int64 words


def query_slice(nq: int, rank: int, world: int) -> Tuple[int, int]:
    """[begin, end) of this rank's queries in replica mode."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    return (nq * rank) // world, (nq * (rank + 1)) // world


def all_gather_entries(local: torch.Tensor, world: int, group=None) -> torch.Tensor:
    """The one collective of a range-split batch: [nq, k, 2] int64 per rank ->
    [world, nq, k, 2] on every rank (any equal-shaped tensor per rank ->
    [world, ...])."""
    out = torch.empty((world,) + tuple(local.shape), dtype=local.dtype, device=local.device)
    if world == 1:
        out[0].copy_(local)
        return out
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, local.contiguous(), group=group)
    elif local.device.type == "cpu":   # gloo (CPU tests): list form
        parts = list(out.unbind(0))
        dist.all_gather(parts, local.contiguous(), group=group)
    else:   # gloo with device tensors (multi-process tests on one GPU): via host memory
        host = torch.empty((world,) + tuple(local.shape), dtype=local.dtype)
        dist.all_gather(list(host.unbind(0)), local.cpu(), group=group)
        out.copy_(host)
    return out


class NativeShardEngine:
    """A shard's HIP index (device ``device``) behind the engine interface the
    searcher uses; inputs and outputs are torch tensors on that device."""

    def __init__(self, shard_index, device: int = 0):
        from ._native import NativeIndex
        if not shard_index.is_shard:
            raise ValueError("NativeShardEngine needs a TreeAHIndex.shard(...)")
        self.nat = NativeIndex(shard_index, device=device)
        self.device = torch.device("cuda", device)
        # the C ABI maps a NULL stream to the index's own stream, and torch's
        # default stream handle is NULL: run the native calls on a stream of
        # our own, ordered against the caller's current stream both ways
        self.stream = torch.cuda.Stream(device=self.device)

    def _enter(self, *tensors):
        """The stream the native call runs on: the caller's current stream
        when it is a stream of its own (the library keeps one workspace per
        stream, so batches on different streams run concurrently), else the
        engine's stream, ordered against the caller's both ways."""
        cur = torch.cuda.current_stream(self.device)
        if cur.cuda_stream != 0:
            return cur, cur
        self.stream.wait_stream(cur)
        for t in tensors:
            t.record_stream(self.stream)
        return cur, self.stream

    def shard_width(self, leaves, pre_nn, final_nn, reorder) -> int:
        return self.nat.shard_width(leaves, pre_nn, final_nn, reorder)

    def search_shard(self, queries: torch.Tensor, leaves, pre_nn, final_nn, reorder,
                     out_entries: torch.Tensor) -> None:
        q = queries.contiguous()
        cur, run = self._enter(q, out_entries)
        self.nat.search_shard_device(q.data_ptr(), q.shape[0], leaves, pre_nn, final_nn, reorder,
                                     out_entries.data_ptr(), run.cuda_stream)
        if run is not cur:
            cur.wait_stream(run)

    def merge(self, world, entries: torch.Tensor, nq, leaves, pre_nn, final_nn, reorder):
        idx = torch.empty((nq, final_nn), dtype=torch.int32, device=self.device)
        dst = torch.empty((nq, final_nn), dtype=torch.float32, device=self.device)
        cnt = torch.empty((nq,), dtype=torch.int32, device=self.device)
        ent = entries.contiguous()
        cur, run = self._enter(ent, idx, dst, cnt)
        self.nat.merge_shards_device(world, nq, leaves, pre_nn, final_nn, reorder, ent.data_ptr(),
                                     idx.data_ptr(), dst.data_ptr(), cnt.data_ptr(),
                                     run.cuda_stream)
        if run is not cur:
            cur.wait_stream(run)
        return idx, dst, cnt


class RangeSplitSearcher:
    """``search_batched`` over a range-split index; every rank calls it with
    the same query batch and gets the same (whole-index) result."""

    def __init__(self, engine, world: Optional[int] = None, group=None):
        self.engine = engine
        self.group = group
        self.world = world if world is not None else dist.get_world_size(group)

    def search_batched(self, queries: torch.Tensor, leaves: int, pre_nn: int, final_nn: int,
                       reorder: bool = True):
        nq = int(queries.shape[0])
        k = self.engine.shard_width(leaves, pre_nn, final_nn, reorder)
        local = torch.empty((nq, k, ENTRY_INT64S), dtype=torch.int64, device=queries.device)
        self.engine.search_shard(queries, leaves, pre_nn, final_nn, reorder, local)
        gathered = all_gather_entries(local, self.world, self.group)
        return self.engine.merge(self.world, gathered, nq, leaves, pre_nn, final_nn, reorder)


class SplitBatchSearcher:
    """Strong scaling over replicas: every rank calls ``search_batched`` with
    the same whole batch; rank r searches rows ``query_slice(nq, r, world)``
    with ``search(q_slice) -> (idx, dist, count)`` (device or CPU tensors), the
    slices -- padded to ceil(nq / world) rows, the all-gather's equal shape --
    are gathered in one collective per output, and every rank returns the
    whole batch's (idx [nq, k], dist [nq, k], count [nq]) in query order: the
    1-rank result bit for bit, since each query's search does not depend on
    the others of its batch."""

    def __init__(self, search, rank: int, world: int, group=None):
        self.search = search
        self.rank = rank
        self.world = world
        self.group = group

    def search_batched(self, queries: torch.Tensor):
        nq = int(queries.shape[0])
        b, e = query_slice(nq, self.rank, self.world)
        idx, dst, cnt = self.search(queries[b:e])
        if self.world == 1:
            return idx, dst, cnt
        rows = (nq + self.world - 1) // self.world
        bounds = [query_slice(nq, r, self.world) for r in range(self.world)]

        def gather(t):
            pad = torch.zeros((rows,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
            pad[: t.shape[0]].copy_(t)
            g = all_gather_entries(pad, self.world, self.group)
            return torch.cat([g[r, : hi - lo] for r, (lo, hi) in enumerate(bounds)], 0)

        return gather(idx), gather(dst), gather(cnt)
