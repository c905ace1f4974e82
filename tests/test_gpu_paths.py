"""The search's alternative device paths against the oracle and each other.

These switches select kernels without changing any result (all are read
when a handle is created):

  * SMX_SEED_MFMA -- the per-query seed thresholds from the seed scan
    (seed_scan_kernel + seed_select_kernel: 16-query MFMA tiles over each
    seed leaf, SeedClaims' row budgets) instead of one block per query
    (seed_tau_kernel + pair_scatter_kernel);
  * SMX_NARROW -- 16-slot scan tiles (v_smfmac_i32_16x16x128_i8): 0 none,
    1 by density (a leaf's last <= 16 queries below 32 queries per leaf on
    average, 16-slot tiles only below 16), 2 16-slot tiles only, 3 never the
    16-slot-only mode;
  * SMX_FUSED_WORKLIST=0 / SMX_SERIAL_WORKLIST=0 -- the work list from its
    three launches (as above 4096 leaves), on the seed's stream or on the
    side stream.

Every combination must give the oracle's ids and distance bits
(tree_ah_hybrid_residual.cc:631-846).  The two seed paths rank the same
values (the query's seed leaves in order, kSeedKeys rows in all), so with no
seed leaf dropped (at most kSeedSlots = 64 queries claim one leaf) their
thresholds -- and so the candidates that pass them -- are identical:
mean_candidates must match exactly.  With more queries per leaf than slots,
a dropped leaf only loosens a threshold; results still match the oracle.
"""
import os

import numpy as np
import pytest

from tests.conftest import make_index

pytestmark = pytest.mark.gpu

PATHS = [{"SMX_SEED_MFMA": s, "SMX_NARROW": n} for s in "01" for n in "0123"] + [
    # the work list by its three launches: before the seed on one stream, and
    # on the side stream beside it (the paths above 4096 leaves)
    {"SMX_SEED_MFMA": "0", "SMX_NARROW": "1", "SMX_FUSED_WORKLIST": "0"},
    {"SMX_SEED_MFMA": "0", "SMX_NARROW": "1", "SMX_FUSED_WORKLIST": "0",
     "SMX_SERIAL_WORKLIST": "0"},
]


def _handle(ix, env):
    from scann_amd import _native
    old = {k: os.environ.get(k) for k in env}
    try:
        os.environ.update(env)
        return _native.NativeIndex(ix)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _search(ix, q, env, L, pre, seed, reorder=True):
    nat = _handle(ix, env)
    try:
        nat.set_tuning(candidates_per_query=0, seed_leaves=seed)
        nat.set_profiling(True)
        gi, gd, gc = nat.search_batched(q, L, pre, 10, reorder)
        t = nat.timings()
    finally:
        nat.close()
    return gi, gd, gc, t


def _check(oracle, ix, q, L, pre, seed, reorder=True):
    oi, od, oc = oracle.search(ix, q, L, pre, 10, reorder, oracle.MODE_IDEAL)
    cands = {}
    for env in PATHS:
        gi, gd, gc, t = _search(ix, q, env, L, pre, seed, reorder)
        tag = f"{env} L={L} pre={pre} seed={seed}"
        np.testing.assert_array_equal(gc, oc, err_msg=tag)
        np.testing.assert_array_equal(gi, oi, err_msg=tag)
        np.testing.assert_array_equal(gd.view(np.uint32), od.view(np.uint32), err_msg=tag)
        if len(env) == 2:
            cands[(env["SMX_SEED_MFMA"], env["SMX_NARROW"])] = t["mean_candidates"]
    return cands


@pytest.fixture(scope="module")
def big_leaves():
    """Residual dot product, 100 dims (K = 26), ~4000 rows per leaf: a seed
    leaf's budget spans all four 1024-row chunks of the seed scan."""
    return make_index(n=40000, d=100, leaves=10, seed=21, components=40)


@pytest.mark.parametrize("fix", ["small_dot", "small_l2"])
@pytest.mark.parametrize("seed", [1, 4])
def test_paths_match_oracle_and_each_other(oracle, fix, seed, request):
    ix, db, q = request.getfixturevalue(fix)
    c = _check(oracle, ix, q, 12, 100, seed)
    assert c[("0", "0")] == c[("1", "0")], c   # same thresholds (64 queries: no drops)


@pytest.mark.parametrize("seed,L,pre", [(1, 3, 100), (2, 4, 200), (4, 6, 100)])
def test_paths_with_multi_chunk_seed_leaves(oracle, big_leaves, seed, L, pre):
    ix, db, q = big_leaves
    assert np.diff(ix.leaf_offsets).max() > 3072
    c = _check(oracle, ix, q, L, pre, seed)
    assert c[("0", "0")] == c[("1", "0")], c


def test_paths_with_dropped_seed_leaves(oracle, small_dot):
    """600 queries near 6 base queries: their seed leaves are claimed by ~100
    queries each, past the 64 slots; a query without a slot ranks "no value"
    over that leaf's range and its threshold is looser, never tighter."""
    ix, db, q = small_dot
    rng = np.random.default_rng(5)
    qq = np.repeat(q[:6], 100, axis=0) + rng.normal(0, 1e-3, (600, q.shape[1])).astype(np.float32)
    qq /= np.linalg.norm(qq, axis=1, keepdims=True)
    c = _check(oracle, ix, qq.astype(np.float32), 12, 100, 4)
    assert c[("1", "0")] >= c[("0", "0")], c


def test_paths_without_seed(oracle, small_l2):
    ix, db, q = small_l2
    _check(oracle, ix, q, 12, 100, 0, reorder=False)
