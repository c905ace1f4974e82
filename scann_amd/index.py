"""Host-side representation of a tree-AH (LUT16) index.

This is the data the query path consumes: leaf centers,
the AH codebook, per-leaf member lists with their 4-bit codes, and the float
rows used for exact reordering.  It corresponds to what the reference keeps
inside ``TreeAHHybridResidual`` (``datapoints_by_token_``, the leaf
searchers' packed codes and the partitioner's centers;
scann/tree_x_hybrid/tree_ah_hybrid_residual.h:293-320) and to the assets
``load_searcher`` reads (scann/scann_ops/cc/scann.cc:105-233).

``IndexDesc`` is the ctypes mirror of ``smx_index_desc``
(include/scann_mi355x.h); the oracle's ``orc_index`` has the same layout.
"""
from __future__ import annotations

import ctypes
import dataclasses
from typing import Optional

import numpy as np

METRIC_DOT = 0
METRIC_SQUARED_L2 = 1
METRIC_NAMES = {"dot_product": METRIC_DOT, "squared_l2": METRIC_SQUARED_L2}


class IndexDesc(ctypes.Structure):
    """ctypes mirror of smx_index_desc / orc_index (identical layout)."""

    _fields_ = [
        ("metric", ctypes.c_int32),
        ("dim", ctypes.c_int32),
        ("num_leaves", ctypes.c_int32),
        ("num_blocks", ctypes.c_int32),
        ("dims_per_block", ctypes.c_int32),
        ("residual", ctypes.c_int32),
        ("centers", ctypes.c_void_p),
        ("codebook", ctypes.c_void_p),
        ("leaf_offsets", ctypes.c_void_p),
        ("leaf_members", ctypes.c_void_p),
        ("member_codes", ctypes.c_void_p),
        ("num_datapoints", ctypes.c_uint32),
        ("dataset", ctypes.c_void_p),
        ("spilling_overretrieve_factor", ctypes.c_float),
        ("pad_", ctypes.c_int32),
        # range-split shard (include/scann_mi355x.h); zero for a whole index
        ("is_shard", ctypes.c_int32),
        ("global_topn_shift", ctypes.c_int32),
        ("global_spilled", ctypes.c_int32),
        ("reserved2", ctypes.c_int32),
        ("leaf_row_base", ctypes.c_void_p),
        ("member_rows", ctypes.c_void_p),
    ]


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data


@dataclasses.dataclass
class TreeAHIndex:
    metric: int
    dim: int
    num_blocks: int
    dims_per_block: int
    residual: bool
    centers: np.ndarray          # float32 [L, D]
    codebook: np.ndarray         # float32 [B, 16, dims_per_block]
    leaf_offsets: np.ndarray     # uint64 [L+1]
    leaf_members: np.ndarray     # uint32 [M], ascending within each leaf
    member_codes: np.ndarray     # uint8 [M, B]
    num_datapoints: int
    dataset: Optional[np.ndarray] = None   # float32 [N, D] (exact reorder)
    spilling_overretrieve_factor: float = 2.0
    # range-split shard of a whole index; see shard()
    leaf_row_base: Optional[np.ndarray] = None   # uint32 [L]
    global_topn_shift: int = -1
    global_spilled: bool = False
    member_rows: Optional[np.ndarray] = None     # float32 [M, D]

    def __post_init__(self):
        self.centers = np.ascontiguousarray(self.centers, dtype=np.float32)
        self.codebook = np.ascontiguousarray(self.codebook, dtype=np.float32)
        self.leaf_offsets = np.ascontiguousarray(self.leaf_offsets, dtype=np.uint64)
        self.leaf_members = np.ascontiguousarray(self.leaf_members, dtype=np.uint32)
        self.member_codes = np.ascontiguousarray(self.member_codes, dtype=np.uint8)
        if self.dataset is not None:
            self.dataset = np.ascontiguousarray(self.dataset, dtype=np.float32)
        if self.leaf_row_base is not None:
            self.leaf_row_base = np.ascontiguousarray(self.leaf_row_base, dtype=np.uint32)
        if self.member_rows is not None:
            self.member_rows = np.ascontiguousarray(self.member_rows, dtype=np.float32)
        self.validate()

    @property
    def num_leaves(self) -> int:
        return int(self.centers.shape[0])

    @property
    def num_members(self) -> int:
        return int(self.leaf_members.shape[0])

    @property
    def is_shard(self) -> bool:
        return self.leaf_row_base is not None

    @property
    def disjoint(self) -> bool:
        if self.is_shard:
            return not self.global_spilled
        return self.num_members == self.num_datapoints

    def global_topn_shift_value(self) -> int:
        """GlobalTopNShift (tree_ah_hybrid_residual.h:234-247) of this whole index."""
        if self.is_shard:
            return int(self.global_topn_shift)
        L = self.num_leaves
        if not self.residual or L <= 1:
            return 0
        inner = 32 - int(np.ceil(np.log2(L)))
        return inner if int(self.leaf_sizes().max(initial=0)) <= (1 << inner) else 0

    def shard(self, rank: int, world: int, own_rows: bool = True) -> "TreeAHIndex":
        """Rank `rank` of a `world`-way range split: rows [n*r/W, n*(r+1)/W) of
        every leaf (balanced whatever the query popularity).
        Ties stay the whole index's (leaf << shift | row) through
        leaf_row_base (or are global ids when a leaf exceeds the global top-N
        limit: shift 0, the reference's fallback, tree_ah_hybrid_residual.h:
        234-247).  With own_rows the shard carries only its members' float
        rows for the reorder instead of the dataset (the device finds a
        candidate's row from its tie, or from its global id at shift 0)."""
        if self.is_shard:
            raise ValueError("already a shard")
        if not 0 <= rank < world:
            raise ValueError("rank out of range")
        sizes = self.leaf_sizes()
        lo = (sizes * rank) // world
        hi = (sizes * (rank + 1)) // world
        offs = self.leaf_offsets.astype(np.int64)
        take = np.concatenate([np.arange(offs[l] + lo[l], offs[l] + hi[l]) for l in range(self.num_leaves)]
                              ) if self.num_leaves else np.zeros(0, np.int64)
        take = take.astype(np.int64)
        new_offs = np.concatenate([[0], np.cumsum(hi - lo)]).astype(np.uint64)
        shift = self.global_topn_shift_value()
        members = self.leaf_members[take]
        rows = None
        dataset = self.dataset
        if own_rows and self.dataset is not None:
            rows = self.dataset[members]
            dataset = None
        return TreeAHIndex(
            metric=self.metric, dim=self.dim, num_blocks=self.num_blocks,
            dims_per_block=self.dims_per_block, residual=self.residual, centers=self.centers,
            codebook=self.codebook, leaf_offsets=new_offs, leaf_members=members,
            member_codes=self.member_codes[take], num_datapoints=self.num_datapoints,
            dataset=dataset, spilling_overretrieve_factor=self.spilling_overretrieve_factor,
            leaf_row_base=lo.astype(np.uint32), global_topn_shift=shift,
            global_spilled=not self.disjoint, member_rows=rows)

    def standalone(self) -> "TreeAHIndex":
        """This shard as a whole index of its own: members renumbered
        0..M-1 (member m <-> global id leaf_members[m]) with their float rows
        as the dataset.  Its ties (leaf << shift | row) order every leaf's
        rows as the shard's whole-index ties do, so for a disjoint index the
        shard's local top-k' is this index's top-k' mapped through
        leaf_members; a SOAR shard's spilled copies become distinct members
        (no dedupe).  The per-rank work of a range split as an index the
        oracle and the CPU port can run (bench.py's shard lines)."""
        if not self.is_shard:
            raise ValueError("standalone() is for a shard")
        rows = self.member_rows
        if rows is None:
            if self.dataset is None:
                raise ValueError("the shard has neither member rows nor a dataset")
            rows = self.dataset[self.leaf_members]
        m = self.num_members
        return TreeAHIndex(metric=self.metric, dim=self.dim, num_blocks=self.num_blocks,
                           dims_per_block=self.dims_per_block, residual=self.residual,
                           centers=self.centers, codebook=self.codebook,
                           leaf_offsets=self.leaf_offsets,
                           leaf_members=np.arange(m, dtype=np.uint32),
                           member_codes=self.member_codes, num_datapoints=m, dataset=rows,
                           spilling_overretrieve_factor=self.spilling_overretrieve_factor)

    def leaf_sizes(self) -> np.ndarray:
        return np.diff(self.leaf_offsets).astype(np.int64)

    def validate(self) -> None:
        L, D = self.centers.shape
        if D != self.dim:
            raise ValueError(f"centers dim {D} != dim {self.dim}")
        B, dpb = self.num_blocks, self.dims_per_block
        last = self.dim - dpb * (B - 1)
        if not (0 < last <= dpb):
            raise ValueError(f"{B} blocks of {dpb} dims do not tile dim {self.dim}")
        if self.codebook.shape != (B, 16, dpb):
            raise ValueError(f"codebook shape {self.codebook.shape} != {(B, 16, dpb)}")
        if self.leaf_offsets.shape != (L + 1,) or self.leaf_offsets[0] != 0:
            raise ValueError("leaf_offsets must have num_leaves+1 entries starting at 0")
        if np.any(np.diff(self.leaf_offsets.astype(np.int64)) < 0):
            raise ValueError("leaf_offsets must be non-decreasing")
        M = int(self.leaf_offsets[-1])
        if self.leaf_members.shape != (M,):
            raise ValueError("leaf_members size mismatch")
        if self.member_codes.shape != (M, B):
            raise ValueError("member_codes shape mismatch")
        if M and int(self.member_codes.max()) > 15:
            raise ValueError("codes must be 4-bit (LUT16)")
        if M and int(self.leaf_members.max()) >= self.num_datapoints:
            raise ValueError("member id out of range")
        if self.dataset is not None and self.dataset.shape != (self.num_datapoints, self.dim):
            raise ValueError("dataset shape mismatch")
        if self.leaf_row_base is not None and self.leaf_row_base.shape != (L,):
            raise ValueError("leaf_row_base must have num_leaves entries")
        if self.member_rows is not None and self.member_rows.shape != (M, self.dim):
            raise ValueError("member_rows must be [members, dim]")

    def desc(self) -> IndexDesc:
        """Borrowed-pointer descriptor; keep ``self`` alive while it is used."""
        return IndexDesc(
            metric=self.metric, dim=self.dim, num_leaves=self.num_leaves,
            num_blocks=self.num_blocks, dims_per_block=self.dims_per_block,
            residual=int(bool(self.residual)),
            centers=_ptr(self.centers), codebook=_ptr(self.codebook),
            leaf_offsets=_ptr(self.leaf_offsets), leaf_members=_ptr(self.leaf_members),
            member_codes=_ptr(self.member_codes), num_datapoints=self.num_datapoints,
            dataset=_ptr(self.dataset),
            spilling_overretrieve_factor=float(self.spilling_overretrieve_factor), pad_=0,
            is_shard=int(self.is_shard),
            global_topn_shift=int(self.global_topn_shift) if self.is_shard else 0,
            global_spilled=int(bool(self.global_spilled)) if self.is_shard else 0,
            reserved2=0, leaf_row_base=_ptr(self.leaf_row_base),
            member_rows=_ptr(self.member_rows))

    # -- serialization (own format; reference proto assets are SURVEY §8f-2) --
    def save(self, directory: str) -> None:
        import json
        import os
        os.makedirs(directory, exist_ok=True)
        meta = dict(metric=self.metric, dim=self.dim, num_blocks=self.num_blocks,
                    dims_per_block=self.dims_per_block, residual=bool(self.residual),
                    num_datapoints=self.num_datapoints,
                    spilling_overretrieve_factor=self.spilling_overretrieve_factor,
                    has_dataset=self.dataset is not None)
        with open(os.path.join(directory, "smx_index.json"), "w") as f:
            json.dump(meta, f)
        for name in ("centers", "codebook", "leaf_offsets", "leaf_members", "member_codes"):
            np.save(os.path.join(directory, f"{name}.npy"), getattr(self, name))
        if self.dataset is not None:
            np.save(os.path.join(directory, "dataset.npy"), self.dataset)

    @classmethod
    def load(cls, directory: str) -> "TreeAHIndex":
        import json
        import os
        with open(os.path.join(directory, "smx_index.json")) as f:
            meta = json.load(f)
        arr = {n: np.load(os.path.join(directory, f"{n}.npy"))
               for n in ("centers", "codebook", "leaf_offsets", "leaf_members", "member_codes")}
        ds = np.load(os.path.join(directory, "dataset.npy")) if meta["has_dataset"] else None
        return cls(metric=meta["metric"], dim=meta["dim"], num_blocks=meta["num_blocks"],
                   dims_per_block=meta["dims_per_block"], residual=meta["residual"],
                   num_datapoints=meta["num_datapoints"], dataset=ds,
                   spilling_overretrieve_factor=meta["spilling_overretrieve_factor"], **arr)
