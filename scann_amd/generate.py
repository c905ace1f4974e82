"""On-device generated indexes for BASELINE.json configs 4 and 5.

Config 4 (100M x 96 dot product, 10000 leaves, SOAR, range split over 8
GPUs) and config 5 (Deep1B shape, 1e9 x 96, 50000 leaves, 8-way shard) are
never materialised on the host: every rank generates the rows it owns on
its GPU, tokenizes them against centers every rank trains identically, and
keeps only its shard.

* Rows.  A unit-norm Gaussian mixture drawn by torch's counter-based Philox
  generator, keyed by (seed, 65536-row chunk): any rank regenerates any
  chunk bit for bit without the others.
* Range split.  Rank r of W owns the chunks [C*r/W, C*(r+1)/W), so every
  rank tokenizes with the same GEMM shapes as a single-process build (the
  assignment of a row does not depend on who computes it).  Members are
  sorted by (leaf, global row); the rows of leaf l that rank r holds are a
  contiguous run of the whole leaf's member list, starting at
  leaf_row_base[l] = the leaf's members on ranks < r -- exactly the shard
  layout of TreeAHIndex.shard(), so ties stay the whole index's
  (leaf << shift | row in the full leaf) and the merged result equals the
  unsharded search.
* Per-leaf counts of the other ranks come from an all-gather when
  torch.distributed is initialised, otherwise from a counting pass over
  their rows on this GPU (assign only; nothing kept).
* Centers: k-means (device_builder.kmeans) on the first
  `training_sample_size` rows of the dataset; codebook: per-block k-means
  (device_builder.train_codebook) on the residuals of the first
  `ah_training_sample_size` rows -- the same samples on every rank.
* Tokens, SOAR secondary leaves, the (leaf, row) grouping, residuals and
  codes: the hand-written HIP build kernels (smx_nearest_centers,
  smx_group_by_leaf, smx_gather_residuals, smx_block_encode) -- every step
  of the build runs in them; torch only generates the rows and holds the
  buffers.
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np
import torch

from . import device_builder as dbuild
from .index import METRIC_DOT, TreeAHIndex

CHUNK = 1 << 16


def _mix(seed: int, chunk: int) -> int:
    """splitmix64 of (seed, chunk) -> a 63-bit Philox seed."""
    z = (seed * 0x9E3779B97F4A7C15 + chunk + 1) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return (z ^ (z >> 31)) & 0x7FFFFFFFFFFFFFFF


class GeneratedDataset:
    """Rows of a seeded unit-norm mixture, generated on `device` per chunk."""

    def __init__(self, n: int, dim: int, seed: int, components: int = 4096,
                 spread: float = 0.9, device: Optional[torch.device] = None):
        self.n, self.dim, self.seed = int(n), int(dim), int(seed)
        self.components, self.spread = int(components), float(spread)
        self.device = device or torch.device("cuda")
        g = torch.Generator(device="cpu").manual_seed(_mix(seed, -1 & 0xFFFFFFFF))
        m = torch.randn(self.components, self.dim, generator=g, dtype=torch.float32)
        self.means = (m / m.norm(dim=1, keepdim=True)).to(self.device)
        self.num_chunks = (self.n + CHUNK - 1) // CHUNK

    def chunk(self, c: int) -> torch.Tensor:
        rows = min(CHUNK, self.n - c * CHUNK)
        g = torch.Generator(device=self.device).manual_seed(_mix(self.seed, c))
        z = torch.randint(0, self.components, (rows,), generator=g, device=self.device)
        x = self.means[z] + (self.spread / math.sqrt(self.dim)) * torch.randn(
            rows, self.dim, generator=g, device=self.device, dtype=torch.float32)
        return x / x.norm(dim=1, keepdim=True)

    def rows(self, start: int, count: int) -> torch.Tensor:
        """Rows [start, start + count) (any range; chunks regenerated)."""
        out = torch.empty(count, self.dim, dtype=torch.float32, device=self.device)
        c0, c1 = start // CHUNK, (start + count - 1) // CHUNK if count else -1
        for c in range(c0, c1 + 1):
            x = self.chunk(c)
            lo = max(start, c * CHUNK)
            hi = min(start + count, c * CHUNK + x.shape[0])
            out[lo - start:hi - start] = x[lo - c * CHUNK:hi - c * CHUNK]
        return out

    def queries(self, nq: int, seed: int) -> np.ndarray:
        """A query batch from the same mixture (its own Philox key)."""
        q = GeneratedDataset(nq, self.dim, seed, self.components, self.spread, self.device)
        q.means = self.means
        return q.rows(0, nq).cpu().numpy()

    def chunk_range(self, rank: int, world: int):
        return (self.num_chunks * rank) // world, (self.num_chunks * (rank + 1)) // world


def _assign(x: torch.Tensor, c: torch.Tensor, cn: torch.Tensor) -> torch.Tensor:
    """Nearest center of every row (smx_nearest_centers)."""
    return dbuild.nearest_centers(x, c)


def _soar(x: torch.Tensor, c: torch.Tensor, cn: torch.Tensor, p: torch.Tensor,
          lam: float) -> torch.Tensor:
    """The SOAR secondary leaf of every row, never the primary
    (smx_nearest_centers with the primary centers)."""
    return dbuild.nearest_centers(x, c, primary=p, lam=float(lam))


def _tokens(ds: GeneratedDataset, c0: int, c1: int, c: torch.Tensor, cn: torch.Tensor,
            soar_lambda: Optional[float], keep: bool):
    """(leaf, row) entries of chunks [c0, c1) (int32 leaves, rows as int32
    storage of uint32 ids); per-leaf counts always."""
    L = c.shape[0]
    counts = torch.zeros(L, dtype=torch.int64, device=ds.device)
    leaves, rows = [], []
    for ch in range(c0, c1):
        x = ds.chunk(ch)
        p = _assign(x, c, cn)
        parts = [p]
        if soar_lambda is not None and L > 1:
            parts.append(_soar(x, c, cn, p, float(soar_lambda)))
        rid = torch.arange(ch * CHUNK, ch * CHUNK + x.shape[0], dtype=torch.int64,
                           device=ds.device).to(torch.int32)
        for t in parts:
            counts += torch.bincount(t, minlength=L)
            if keep:
                leaves.append(t)
                rows.append(rid)
    if keep:
        if not leaves:   # a rank without chunks (n < world chunks)
            e = torch.zeros(0, dtype=torch.int32, device=ds.device)
            return counts, e, e.clone()
        return counts, torch.cat(leaves), torch.cat(rows)
    return counts, None, None


def build_generated_shard(ds: GeneratedDataset, num_leaves: int, rank: int = 0, world: int = 1,
                          *, metric: int = METRIC_DOT, dims_per_block: int = 2,
                          soar_lambda: Optional[float] = None, overretrieve_factor: float = 2.0,
                          training_sample_size: int = 250_000, training_iterations: int = 8,
                          ah_training_sample_size: int = 100_000, ah_training_iterations: int = 8,
                          seed: int = 0, counts_from_all_ranks: bool = True,
                          log=None) -> TreeAHIndex:
    """Rank `rank`'s shard of the generated dataset's tree-AH index (world = 1:
    the whole index, not a shard).  With counts_from_all_ranks=False and no
    process group, the shard skips the counting pass over the other ranks'
    rows: leaf_row_base is then exact only for rank 0 and the global top-N
    shift is taken from this rank's leaf sizes scaled by `world`."""
    import torch.distributed as dist
    dev = ds.device
    say = log or (lambda m: None)
    dim = ds.dim
    residual = metric == METRIC_DOT
    # partitioner: the same sample on every rank
    samp = ds.rows(0, min(training_sample_size, ds.n))
    c = dbuild.kmeans(samp, num_leaves, training_iterations, seed)
    say(f"centers: k-means {num_leaves} on {samp.shape[0]} rows")
    del samp
    centers = c.cpu().numpy()
    cn = None
    L = centers.shape[0]
    num_blocks = int(math.ceil(dim / dims_per_block))
    # codebook: residuals of the first rows' primary leaves
    asamp = ds.rows(0, min(ah_training_sample_size, ds.n))
    ap = _assign(asamp, c, cn)
    ares = dbuild.gather_residuals(asamp, torch.arange(asamp.shape[0], dtype=torch.int32,
                                                       device=dev), ap,
                                   c if residual else None)
    cb = dbuild.train_codebook(ares, num_blocks, dims_per_block, ah_training_iterations,
                               seed + 2)
    codebook = cb.cpu().numpy()
    say(f"codebook: {num_blocks} blocks x 16 on {asamp.shape[0]} residuals")
    del asamp, ap, ares

    c0, c1 = ds.chunk_range(rank, world)
    counts, leaves, rows = _tokens(ds, c0, c1, c, cn, soar_lambda, keep=True)
    say(f"rank {rank}/{world}: chunks [{c0}, {c1}) tokenized, {int(leaves.numel())} members")
    if world == 1:
        before = torch.zeros_like(counts)
        total = counts
    elif dist.is_available() and dist.is_initialized():
        allc = [torch.empty_like(counts) for _ in range(world)]
        dist.all_gather(allc, counts)
        allc = torch.stack(allc)
        before = allc[:rank].sum(0)
        total = allc.sum(0)
    elif counts_from_all_ranks:
        before = torch.zeros_like(counts)
        total = counts.clone()
        for r in range(world):
            if r == rank:
                continue
            rc, _, _ = _tokens(ds, *ds.chunk_range(r, world), c, cn, soar_lambda, keep=False)
            total += rc
            if r < rank:
                before += rc
        say("per-leaf counts of the other ranks: counting pass done")
    else:
        before = torch.zeros_like(counts)
        total = counts * world

    # members by (leaf, row): smx_group_by_leaf
    _, rows, leaves = dbuild.group_by_leaf(leaves, rows, L)
    offsets = np.zeros(L + 1, np.uint64)
    offsets[1:] = np.cumsum(counts.cpu().numpy())
    spilled = soar_lambda is not None and L > 1
    inner = 32 - int(math.ceil(math.log2(L))) if L > 1 else 32
    shift = inner if (residual and L > 1 and int(total.max()) <= (1 << inner)) else 0

    # the members' float rows and codes (nearest codebook center per block)
    m = rows.numel()
    row0 = c0 * CHUNK
    nrows = min(c1 * CHUNK, ds.n) - row0
    x_all = ds.rows(row0, nrows)
    codes = np.empty((m, num_blocks), np.uint8)
    member_rows = np.empty((m, dim), np.float32)
    step = 1 << 23
    for s0 in range(0, m, step):
        rr, ll = rows[s0:s0 + step], leaves[s0:s0 + step]
        xr = dbuild.gather_residuals(x_all, rr, None, None, row_base=row0)
        member_rows[s0:s0 + rr.numel()] = xr.cpu().numpy()
        res = dbuild.gather_residuals(x_all, rr, ll, c, row_base=row0) if residual else xr
        codes[s0:s0 + rr.numel()] = dbuild.block_encode(res, cb).cpu().numpy()
        del xr, res
    del x_all
    say(f"codes: {m} members encoded; largest leaf {int(total.max())} (whole index"
        f"{', estimated' if world > 1 and not counts_from_all_ranks else ''}), shift {shift}")
    members = rows.cpu().numpy().view(np.uint32)
    if world == 1:
        dataset = np.empty((ds.n, dim), np.float32)
        dataset[members] = member_rows   # a SOAR copy writes the same row twice
        return TreeAHIndex(metric=metric, dim=dim, num_blocks=num_blocks,
                           dims_per_block=dims_per_block, residual=residual, centers=centers,
                           codebook=codebook, leaf_offsets=offsets, leaf_members=members,
                           member_codes=codes, num_datapoints=ds.n, dataset=dataset,
                           spilling_overretrieve_factor=float(overretrieve_factor))
    # shift 0 (a leaf above the global top-N limit, the reference's fallback
    # to global-id ties): the shard still reorders from its own rows (the
    # device maps a candidate's global id to its member slot)
    return TreeAHIndex(metric=metric, dim=dim, num_blocks=num_blocks,
                       dims_per_block=dims_per_block, residual=residual, centers=centers,
                       codebook=codebook, leaf_offsets=offsets, leaf_members=members,
                       member_codes=codes, num_datapoints=ds.n,
                       spilling_overretrieve_factor=float(overretrieve_factor),
                       leaf_row_base=before.cpu().numpy().astype(np.uint32),
                       global_topn_shift=shift, global_spilled=spilled,
                       member_rows=member_rows)
