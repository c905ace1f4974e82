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
