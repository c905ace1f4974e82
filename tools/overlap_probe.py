"""Probe: do two query batches in flight on two streams raise throughput?

    python tools/overlap_probe.py [--steps 200] [--config glove]

Builds the bench index, then times K batches (a) on one handle and stream,
back to back (the bench's step), and (b) alternating between H handles of
the same index, each on its own stream with its own query/output buffers, so
that one batch's latency-bound kernels can run beside the other's.
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--config", default="glove")
    ap.add_argument("--handles", type=int, default=2)
    args = ap.parse_args()
    bench.CFG = bench.CONFIGS[args.config]
    bench.LEAVES, bench.LEAVES_TO_SEARCH = bench.CFG["leaves"], bench.CFG["leaves_to_search"]
    from scann_amd import _native
    db, _, ix = bench.build_index(bench.CFG["n"], seed=bench.CFG["seed"])
    q = bench.queries_for_rank(db.shape[1], 0)
    dev = torch.device("cuda", 0)
    H = args.handles
    nats = [_native.NativeIndex(ix, device=0) for _ in range(H)]
    streams = [torch.cuda.Stream() for _ in range(H)]
    qd = [torch.from_numpy(q).to(dev) for _ in range(H)]
    outs = [(torch.zeros((bench.NQ, 10), dtype=torch.int32, device=dev),
             torch.zeros((bench.NQ, 10), dtype=torch.float32, device=dev),
             torch.zeros(bench.NQ, dtype=torch.int32, device=dev)) for _ in range(H)]

    def step(i, h, s):
        o = outs[h]
        nats[h].search_batched_device(qd[h].data_ptr(), bench.NQ, bench.LEAVES_TO_SEARCH,
                                      bench.PRE_NN, 10, True, o[0].data_ptr(), o[1].data_ptr(),
                                      o[2].data_ptr(), stream=ctypes_stream(s))

    def ctypes_stream(s):
        import ctypes
        return ctypes.c_void_p(s.cuda_stream)

    def timed(nh):
        for i in range(10):
            step(i, i % nh, streams[i % nh])
        torch.cuda.synchronize()
        t = time.perf_counter()
        for i in range(args.steps):
            step(i, i % nh, streams[i % nh])
        torch.cuda.synchronize()
        return (time.perf_counter() - t) * 1e3 / args.steps

    res = {}
    for rep in range(2):
        for nh in sorted({1, 2, H}):
            res.setdefault(nh, []).append(timed(nh))
    ref = outs[0][0].cpu().numpy()
    same = all(np.array_equal(ref, o[0].cpu().numpy()) for o in outs)
    for nh, v in res.items():
        print(f"handles/streams in flight {nh}: ms per batch {['%.4f' % x for x in v]} "
              f"-> {bench.NQ / min(v) * 1e3 / 1e6:.3f}M QPS", flush=True)
    print("results identical across handles:", same)
    for n in nats:
        n.close()


if __name__ == "__main__":
    main()
