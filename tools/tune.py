"""Stage timings of the glove-shaped search for a grid of tuning knobs.

    python tools/tune.py            (on the GPU box)
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# the scan variants other than 0 exist only in the diagnostic library
os.environ.setdefault("SMX_LIB", os.path.join(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))), "scann_amd", "lib", "libscann_mi355x_time.so"))
import torch  # noqa: E402

from bench import LEAVES_TO_SEARCH, NQ, PRE_NN, FINAL_NN, build_index  # noqa: E402
from scann_amd import _native  # noqa: E402


def main():
    db, q, ix = build_index(1_183_514, seed=2)
    nat = _native.NativeIndex(ix)
    nat.set_profiling(True)
    qd = torch.from_numpy(q).cuda()
    oi = torch.zeros((NQ, FINAL_NN), dtype=torch.int32, device="cuda")
    od = torch.zeros((NQ, FINAL_NN), dtype=torch.float32, device="cuda")
    grid = [tuple(int(x) for x in g.split(",")) for g in sys.argv[1:]] or [
        (4096, 2, 0, 32), (4096, 2, 2, 32), (4096, 2, 3, 32), (4096, 2, 2, 16), (4096, 2, 3, 64)]
    for cap, seed, variant, chunk in grid:
        nat.set_tuning(cap, seed, variant, chunk)
        acc = {}
        steps = 10
        for i in range(steps + 2):
            nat.search_batched_device(qd.data_ptr(), NQ, LEAVES_TO_SEARCH, PRE_NN, FINAL_NN, True,
                                      oi.data_ptr(), od.data_ptr(), None)
            t = nat.timings()
            if i >= 2:
                for k, v in t.items():
                    acc[k] = acc.get(k, 0.0) + float(v) / steps
        nat.set_profiling(False)
        for _ in range(3):
            nat.search_batched_device(qd.data_ptr(), NQ, LEAVES_TO_SEARCH, PRE_NN, FINAL_NN, True,
                                      oi.data_ptr(), od.data_ptr(), None)
        torch.cuda.synchronize()
        tw = time.perf_counter()
        for _ in range(50):
            nat.search_batched_device(qd.data_ptr(), NQ, LEAVES_TO_SEARCH, PRE_NN, FINAL_NN, True,
                                      oi.data_ptr(), od.data_ptr(), None)
        torch.cuda.synchronize()
        wall_ms = (time.perf_counter() - tw) * 1000.0 / 50
        nat.set_profiling(True)
        mfma_tops = acc["scan_item_tiles"] * 26 * 65536 / (acc["scan_ms"] * 1e-3) / 1e12
        print(f"var={variant} chunk={chunk:3d} cap={cap:5d} seed={seed:2d} total={acc['total_ms']:.3f} part={acc['partition_ms']:.3f} "
              f"lut={acc['lut_ms']:.3f} inv={acc['invert_ms']:.3f} seed={acc['seed_scan_ms']:.3f} "
              f"scan={acc['scan_ms']:.3f} sel={acc['select_ms']:.3f} retries={acc['overflow_retries']:.1f} "
              f"cand_mean={acc['mean_candidates']:.0f} cand_max={acc['max_candidates']:.0f} "
              f"item_tiles={acc['scan_item_tiles']:.0f} mfma={mfma_tops:.0f}TOPS wall={wall_ms:.3f}ms "
              f"wgs={acc['scan_workgroups']:.0f}", flush=True)


if __name__ == "__main__":
    main()
