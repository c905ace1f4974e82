"""Diagnostic (GPU box): the per-query seed threshold paths on one shard of
tests/test_gpu_shards.py::_oversized_leaf_index viewed as a standalone index:
pre-reorder lists against the oracle for seed_leaves 0/1/2/4."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import binding as oracle  # noqa: E402
from scann_amd import _native  # noqa: E402
from tests.test_gpu_shards import _oversized_leaf_index  # noqa: E402


def main():
    oracle.build()
    ix, q, db = _oversized_leaf_index(False)
    for r in (3, 0):
        view = ix.shard(r, 4).standalone()
        nat = _native.NativeIndex(view)
        oi, od, oc = oracle.search_pre_reorder(view, q, 8, 60, oracle.MODE_IDEAL)
        for seed in (0, 1, 2, 4):
            nat.set_tuning(0, seed)
            gi, gd, gc = nat.search_pre_reorder(q, 8, 60)
            bad = [i for i in range(q.shape[0]) if gc[i] != oc[i] or
                   not np.array_equal(gi[i, :gc[i]], oi[i, :oc[i]])]
            print(f"shard {r} seed {seed}: {len(bad)} queries differ {bad[:8]} "
                  f"(counts gpu {[int(gc[i]) for i in bad[:4]]} oracle {[int(oc[i]) for i in bad[:4]]})",
                  flush=True)
        nat.close()


if __name__ == "__main__":
    main()
