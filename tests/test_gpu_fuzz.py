"""GPU parity over seeded random configurations.

Each case draws its index and search parameters from its own seed: dataset
size and dimension, dims per block (so the scan's K instantiation, odd block
counts included), metric, residual or not, SOAR spilling or disjoint leaves,
leaves_to_search (up to past the leaf count), pre_reorder_nn / final_nn
(1 up to past the candidates available), reorder on or off, batch size.  The
bar is the other parity tests': ids, counts and distance bits equal to the
oracle's ideal mode (oracle/ restates the reference's search; see
tests/test_gpu_parity.py for the per-stage tests this widens).
"""
import math

import numpy as np
import pytest

N_CASES = 40


def draw(case):
    rng = np.random.default_rng(7000 + case)
    d = int(rng.choice([8, 12, 20, 31, 32, 50, 64, 100, 128]))
    dpbs = [p for p in (1, 2, 3, 4) if math.ceil(d / p) <= 64]
    dpb = int(rng.choice(dpbs))
    metric = int(rng.integers(2))
    p = dict(
        n=int(rng.integers(400, 7000)), d=d, dpb=dpb, metric=metric,
        leaves=int(rng.integers(1, 70)),
        residual=bool(rng.integers(2)) if metric == 0 else False,
        soar=bool(rng.random() < 0.35),
        nq=int(rng.choice([1, 3, 33, 64, 129])),
        pre=int(rng.choice([1, 7, 40, 100, 300])),
        reorder=bool(rng.integers(2)),
        seed=int(rng.integers(1, 1000)),
    )
    p["L"] = int(rng.integers(1, p["leaves"] + 4))
    p["final"] = int(min(p["pre"], rng.choice([1, 5, 10, 33])))
    return p


def build(p):
    from scann_amd import index_builder, synthetic
    norm = p["metric"] == 0
    comps = max(2, min(48, p["n"] // 60))
    db = synthetic.mixture(p["n"], p["d"], comps, 0.9, p["seed"], normalize=norm)
    q = synthetic.mixture(p["nq"], p["d"], comps, 0.9, p["seed"] + 100, normalize=norm,
                          means_seed=p["seed"])
    ix = index_builder.build_tree_ah(db, p["metric"], p["leaves"], p["dpb"],
                                     training_iterations=4, ah_training_iterations=4,
                                     residual=p["residual"],
                                     soar_lambda=1.5 if p["soar"] else None, seed=p["seed"])
    return ix, q


def test_draws_cover_the_space():
    ps = [draw(c) for c in range(N_CASES)]
    assert {p["metric"] for p in ps} == {0, 1}
    assert {p["soar"] for p in ps} == {False, True}
    assert {p["reorder"] for p in ps} == {False, True}
    assert any(p["L"] > p["leaves"] for p in ps)
    assert any(math.ceil(p["d"] / p["dpb"]) % 2 for p in ps)   # odd block counts


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(N_CASES))
def test_random_configuration_matches_oracle(oracle, case):
    from scann_amd import _native
    p = draw(case)
    ix, q = build(p)
    nat = _native.NativeIndex(ix)
    gi, gd, gc = nat.search_pre_reorder(q, p["L"], p["pre"])
    oi, od, oc = oracle.search_pre_reorder(ix, q, p["L"], p["pre"], oracle.MODE_IDEAL)
    np.testing.assert_array_equal(gc, oc, err_msg=str(p))
    np.testing.assert_array_equal(gi, oi, err_msg=str(p))
    np.testing.assert_array_equal(gd.view(np.uint32), od.view(np.uint32), err_msg=str(p))
    gi, gd, gc = nat.search_batched(q, p["L"], p["pre"], p["final"], p["reorder"])
    oi, od, oc = oracle.search(ix, q, p["L"], p["pre"], p["final"], p["reorder"],
                               oracle.MODE_IDEAL)
    np.testing.assert_array_equal(gc, oc, err_msg=str(p))
    np.testing.assert_array_equal(gi, oi, err_msg=str(p))
    np.testing.assert_array_equal(gd.view(np.uint32), od.view(np.uint32), err_msg=str(p))


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(0, N_CASES, 3))
def test_random_configuration_sharded_and_sub_batched(oracle, case):
    """The same draws through the range-split path (W = 2..4 shards of the
    leaves, their lists merged on the device; shard rows or dataset rows) and
    through the device entry point with a leaf-slot budget that forces
    sub-batches of ~1/3 of the batch: the oracle's whole-index results."""
    import os
    import torch
    from scann_amd import _native
    from scann_amd.distributed import NativeShardEngine
    p = draw(case)
    ix, q = build(p)
    rng = np.random.default_rng(case)
    oi, od, oc = oracle.search(ix, q, p["L"], p["pre"], p["final"], p["reorder"],
                               oracle.MODE_IDEAL)
    qd = torch.from_numpy(q).cuda()
    nq = q.shape[0]
    world = int(min(ix.num_leaves, rng.integers(2, 5)))
    if world >= 2:
        own = bool(rng.integers(2))
        engines = [NativeShardEngine(ix.shard(r, world, own_rows=own), device=0)
                   for r in range(world)]
        k = engines[0].shard_width(p["L"], p["pre"], p["final"], p["reorder"])
        entries = torch.empty((world, nq, k, 2), dtype=torch.int64, device="cuda")
        for r, e in enumerate(engines):
            e.search_shard(qd, p["L"], p["pre"], p["final"], p["reorder"], entries[r])
        idx, dst, cnt = engines[0].merge(world, entries, nq, p["L"], p["pre"], p["final"],
                                         p["reorder"])
        torch.cuda.synchronize()
        np.testing.assert_array_equal(cnt.cpu().numpy(), oc, err_msg=str(p))
        np.testing.assert_array_equal(idx.cpu().numpy().astype(np.uint32), oi, err_msg=str(p))
        np.testing.assert_array_equal(dst.cpu().numpy().view(np.uint32), od.view(np.uint32),
                                      err_msg=str(p))
    budget = str(max(1, ix.num_leaves * max(1, -(-nq // 3))))
    old = os.environ.get("SMX_LEAF_SLOT_BUDGET")
    os.environ["SMX_LEAF_SLOT_BUDGET"] = budget
    try:
        nat = _native.NativeIndex(ix)
    finally:
        if old is None:
            os.environ.pop("SMX_LEAF_SLOT_BUDGET")
        else:
            os.environ["SMX_LEAF_SLOT_BUDGET"] = old
    try:
        f = p["final"]
        di = torch.zeros((nq, f), dtype=torch.int32, device="cuda")
        dd = torch.zeros((nq, f), dtype=torch.float32, device="cuda")
        dc = torch.zeros(nq, dtype=torch.int32, device="cuda")
        nat.search_batched_device(qd.data_ptr(), nq, p["L"], p["pre"], p["final"], p["reorder"],
                                  di.data_ptr(), dd.data_ptr(), dc.data_ptr())
        torch.cuda.synchronize()
        np.testing.assert_array_equal(dc.cpu().numpy(), oc, err_msg=str(p))
        np.testing.assert_array_equal(di.cpu().numpy().astype(np.uint32), oi, err_msg=str(p))
        np.testing.assert_array_equal(dd.cpu().numpy().view(np.uint32), od.view(np.uint32),
                                      err_msg=str(p))
    finally:
        nat.close()


def draw_large(case):
    """Batches of hundreds to thousands of queries over tens of thousands of
    rows: many query tiles per leaf, 16- and 32-slot items, several segments
    per workgroup and candidate lists past their first capacity."""
    rng = np.random.default_rng(9100 + case)
    d = int(rng.choice([32, 64, 96, 100, 128]))
    metric = int(rng.integers(2))
    p = dict(n=int(rng.integers(20000, 60000)), d=d, dpb=2, metric=metric,
             leaves=int(rng.integers(40, 400)), residual=metric == 0 and bool(rng.integers(2)),
             soar=bool(rng.random() < 0.3), nq=int(rng.choice([300, 1000, 2500])),
             pre=int(rng.choice([10, 100, 250])), reorder=bool(rng.integers(2)),
             seed=int(rng.integers(1, 1000)))
    p["L"] = int(rng.integers(1, max(2, p["leaves"] // 4)))
    p["final"] = int(min(p["pre"], 10))
    return p


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(8))
def test_random_large_batch_matches_oracle(oracle, case):
    from scann_amd import _native
    p = draw_large(case)
    ix, q = build(p)
    nat = _native.NativeIndex(ix)
    gi, gd, gc = nat.search_batched(q, p["L"], p["pre"], p["final"], p["reorder"])
    oi, od, oc = oracle.search(ix, q, p["L"], p["pre"], p["final"], p["reorder"],
                               oracle.MODE_IDEAL)
    np.testing.assert_array_equal(gc, oc, err_msg=str(p))
    np.testing.assert_array_equal(gi, oi, err_msg=str(p))
    np.testing.assert_array_equal(gd.view(np.uint32), od.view(np.uint32), err_msg=str(p))
