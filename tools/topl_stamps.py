"""Phase timeline of the sampled top-L kernel (topl_sample_kernel) on a
Deep1B-shaped partition (50000 leaves, 96 dims, 1000 queries; diagnostic
build with phase stamps, see tools/phase_stamps.py).

    python tools/phase_stamps.py build      (here)
    python tools/topl_stamps.py [L]          (on the GPU box)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LIB = os.path.join(ROOT, "scann_amd", "lib", "libscann_mi355x_time.so")
PHASES = ["samples", "kth of samples", "compact", "rank", "out+atomics+lut"]


def main():
    L = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    os.environ["SMX_LIB"] = LIB
    path = "/tmp/smx_topl_phase.bin"
    os.environ["SMX_PHASE_FILE"] = path
    import torch
    from scann_amd import _native
    from scann_amd.index import TreeAHIndex
    nl, dim, n, nq = 50000, 96, 400000, 1000
    rng = np.random.default_rng(3)
    centers = rng.standard_normal((nl, dim)).astype(np.float32)
    labels = np.sort(rng.integers(0, nl, n))
    counts = np.bincount(labels, minlength=nl)
    offsets = np.zeros(nl + 1, np.uint64)
    offsets[1:] = np.cumsum(counts)
    nb = dim // 2
    ix = TreeAHIndex(metric=0, dim=dim, num_blocks=nb, dims_per_block=2, residual=True,
                     centers=centers,
                     codebook=(0.3 * rng.standard_normal((nb, 16, 2))).astype(np.float32),
                     leaf_offsets=offsets, leaf_members=np.arange(n, dtype=np.uint32),
                     member_codes=rng.integers(0, 16, (n, nb)).astype(np.uint8),
                     num_datapoints=n, dataset=rng.standard_normal((n, dim)).astype(np.float32))
    q = torch.from_numpy(rng.standard_normal((nq, dim)).astype(np.float32)).cuda()
    nat = _native.NativeIndex(ix)
    oi = torch.zeros((nq, 10), dtype=torch.int32, device="cuda")
    od = torch.zeros((nq, 10), dtype=torch.float32, device="cuda")
    for _ in range(4):
        nat.search_batched_device(q.data_ptr(), nq, L, 100, 10, True, oi.data_ptr(),
                                  od.data_ptr(), None)
    torch.cuda.synchronize()
    t = np.fromfile(path, dtype=np.uint64).reshape(3, 4096, 8)[0, :nq].astype(np.int64)
    n = len(PHASES) + 1
    ok = (t[:, :n] > 0).all(1)
    t = t[ok][:, :n]
    t0 = t[:, 0].min()
    st = (t[:, 0] - t0) / 100.0
    en = (t[:, n - 1] - t0) / 100.0
    print(f"topl_sample L={L}: {len(t)} queries, span {(t[:, n - 1].max() - t0) / 100.0:.1f} us; "
          f"start p50 {np.median(st):.1f} max {st.max():.1f}; end p50 {np.median(en):.1f} "
          f"max {en.max():.1f}")
    for i, ph in enumerate(PHASES):
        d = (t[:, i + 1] - t[:, i]) / 100.0
        print(f"    {ph:18s} p50 {np.median(d):6.2f} p90 {np.percentile(d, 90):6.2f} "
              f"max {d.max():6.2f} us")


if __name__ == "__main__":
    main()
