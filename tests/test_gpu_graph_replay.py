"""Repeated calls with new query contents in the same device buffers: the
first pass is captured once per call shape (hipGraph) and replayed.  Every
call must see its own batch: results are compared with the oracle (ideal
mode) batch by batch, for graph replays and for eager launches, with the
work list built either way."""
import os

import numpy as np
import pytest

from tests.conftest import make_index

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def medium():
    return make_index(n=60000, d=32, leaves=120, seed=21, components=200)


# eager (the default), graph replay; the work list from the fused seed-launch blocks (the
# default at <= 4096 leaves) and from the side-stream fork/join path
@pytest.mark.parametrize("env", [{}, {"SMX_GRAPH": "1"}, {"SMX_FUSED_WORKLIST": "0"},
                                 {"SMX_FUSED_WORKLIST": "0", "SMX_GRAPH": "1"}])
def test_replays_see_new_queries(oracle, medium, env):
    from scann_amd import _native, synthetic
    ix, db, _ = medium
    old = {k: os.environ.get(k) for k in ("SMX_GRAPH", "SMX_NO_GRAPH", "SMX_FUSED_WORKLIST")}
    try:
        for k in old:
            os.environ.pop(k, None)
        os.environ.update(env)
        n = _native.NativeIndex(ix)   # the switches are read at handle creation
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    try:
        for b in range(5):
            q = synthetic.mixture(1000, ix.dim, 200, 0.9, seed=500 + b, means_seed=21)
            gi, gd, gc = n.search_batched(q, 12, 100, 10, True)
            oi, od, oc = oracle.search(ix, q, 12, 100, 10, True, oracle.MODE_IDEAL,
                                       min(16, os.cpu_count() or 1))
            np.testing.assert_array_equal(gi, oi, err_msg=f"batch {b}")
            np.testing.assert_array_equal(gd.view(np.uint32), od.view(np.uint32))
    finally:
        n.close()
