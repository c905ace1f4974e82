"""Batches in flight on several streams of one handle (one workspace per
stream, smx_searcher.hip StreamSlot): every batch's result equals the same
batch searched alone and the oracle, whatever the interleaving -- two to
six streams (a fifth and sixth reuse the oldest slots after waiting for
their work), batches of different shapes on different streams, and the
profiling mode that times the scan launches of calls in flight."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(nat, qd, shapes, streams, outs):
    for i, (L, pre, fin) in enumerate(shapes):
        s = streams[i % len(streams)]
        o = outs[i]
        nat.search_batched_device(qd.data_ptr(), qd.shape[0], L, pre, fin, True, o[0].data_ptr(),
                                  o[1].data_ptr(), o[2].data_ptr(),
                                  stream=ctypes.c_void_p(s.cuda_stream))


@pytest.mark.parametrize("n_streams", [2, 3, 6])
def test_batches_in_flight_match_alone_and_oracle(oracle, small_dot, n_streams):
    from scann_amd import _native
    ix, db, q = small_dot
    nat = _native.NativeIndex(ix)
    qd = torch.from_numpy(q).cuda()
    # alternating shapes, so that slots hold workspaces of different sizes
    shapes = [(12, 100, 10), (6, 40, 10), (20, 60, 5), (12, 100, 10)] * 3
    streams = [torch.cuda.Stream() for _ in range(n_streams)]
    outs = [(torch.zeros((q.shape[0], fin), dtype=torch.int32, device="cuda"),
             torch.zeros((q.shape[0], fin), dtype=torch.float32, device="cuda"),
             torch.zeros(q.shape[0], dtype=torch.int32, device="cuda"))
            for (_, _, fin) in shapes]
    torch.cuda.synchronize()
    _run(nat, qd, shapes, streams, outs)
    torch.cuda.synchronize()
    ref = {}
    for (L, pre, fin), o in zip(shapes, outs):
        if (L, pre, fin) not in ref:
            ref[(L, pre, fin)] = oracle.search(ix, q, L, pre, fin, True, oracle.MODE_IDEAL)
        oi, od, oc = ref[(L, pre, fin)]
        np.testing.assert_array_equal(o[2].cpu().numpy(), oc)
        np.testing.assert_array_equal(o[0].cpu().numpy().astype(np.uint32), oi)
        np.testing.assert_array_equal(o[1].cpu().numpy().view(np.uint32), od.view(np.uint32))
    nat.close()


def test_scan_launch_timing_in_flight(small_dot):
    """Profiling mode 2: an event pair around every scan launch of calls in
    flight, read after the caller synchronises."""
    from scann_amd import _native
    ix, db, q = small_dot
    nat = _native.NativeIndex(ix)
    qd = torch.from_numpy(q).cuda()
    streams = [torch.cuda.Stream() for _ in range(3)]
    shapes = [(12, 100, 10)] * 9
    outs = [(torch.zeros((q.shape[0], 10), dtype=torch.int32, device="cuda"),
             torch.zeros((q.shape[0], 10), dtype=torch.float32, device="cuda"),
             torch.zeros(q.shape[0], dtype=torch.int32, device="cuda")) for _ in shapes]
    torch.cuda.synchronize()
    nat.set_profiling(2)
    _run(nat, qd, shapes, streams, outs)
    torch.cuda.synchronize()
    t = nat.timings()
    nat.set_profiling(False)
    assert t["scan_launches"] == len(shapes)
    assert 0.0 < t["scan_ms_mode2"] < 100.0
    nat.close()
