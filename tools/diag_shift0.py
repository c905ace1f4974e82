"""Diagnostic (GPU box): the shards of an index without the global top-N path
(tests/test_gpu_shards.py::_oversized_leaf_index) -- each shard's local list
from the device against the oracle's exact top-k' of the shard's rows."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import binding as oracle  # noqa: E402
from scann_amd.distributed import NativeShardEngine  # noqa: E402
from scann_amd.index import TreeAHIndex  # noqa: E402
from tests.test_gpu_shards import _oversized_leaf_index  # noqa: E402


def main():
    oracle.build()
    spilled = len(sys.argv) > 1 and sys.argv[1] == "1"
    ix, q, db = _oversized_leaf_index(spilled)
    world, L, pre, fin = 4, 8, 60, 10
    qd = torch.from_numpy(q).cuda()
    for r in range(world):
        sh = ix.shard(r, world)
        own = TreeAHIndex(metric=ix.metric, dim=ix.dim, num_blocks=ix.num_blocks,
                          dims_per_block=ix.dims_per_block, residual=ix.residual,
                          centers=ix.centers, codebook=ix.codebook, leaf_offsets=sh.leaf_offsets,
                          leaf_members=sh.leaf_members, member_codes=sh.member_codes,
                          num_datapoints=ix.num_datapoints, dataset=db,
                          leaf_row_base=sh.leaf_row_base, global_topn_shift=0,
                          global_spilled=spilled)
        eng = NativeShardEngine(sh)
        k = eng.shard_width(L, pre, fin, True)
        ent = torch.empty((q.shape[0], k, 2), dtype=torch.int64, device="cuda")
        eng.search_shard(qd, L, pre, fin, True, ent)
        torch.cuda.synchronize()
        e = ent.cpu().numpy().view(np.uint64)
        pi, pd, pc = oracle.search_pre_reorder(own, q, L, k, oracle.MODE_IDEAL)
        bad = 0
        for i in range(q.shape[0]):
            keys = e[i, :, 0]
            ok = keys != np.uint64(0xFFFFFFFFFFFFFFFF)
            gid = (e[i, ok, 1] & np.uint64(0xFFFFFFFF)).astype(np.uint32)
            tie = (keys[ok] & np.uint64(0xFFFFFFFF)).astype(np.uint32)
            want = pi[i, :pc[i]]
            if len(gid) != pc[i] or set(gid.tolist()) != set(want.tolist()):
                bad += 1
                if bad <= 3:
                    print(f"shard {r} query {i}: device {len(gid)} entries, oracle {pc[i]}; "
                          f"missing {sorted(set(want.tolist()) - set(gid.tolist()))[:8]} "
                          f"extra {sorted(set(gid.tolist()) - set(want.tolist()))[:8]} "
                          f"tie==gid {bool(np.all(tie == gid))}")
        print(f"shard {r}: {bad} of {q.shape[0]} queries differ", flush=True)
        eng.nat.close()


if __name__ == "__main__":
    main()
