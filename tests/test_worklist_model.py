"""The scan's work list (tests/worklist_model.py restates the device code):
every scan workgroup's static share is covered by real work items, and every
tile of every (leaf, query tile) item is scanned exactly once, whatever the
leaf sizes and query counts (empty leaves, leaves without queries, a single
pair, totals smaller than the grid, leaves larger than a chunk)."""
import numpy as np
import pytest

import worklist_model as wm


@pytest.mark.parametrize("qtile", [32, 64])
@pytest.mark.parametrize("seed", range(6))
def test_shares_cover_items_exactly_once(seed, qtile):
    rng = np.random.default_rng(seed)
    nl = int(rng.integers(1, 300))
    sizes = rng.integers(0, 3000, nl)
    sizes[rng.random(nl) < 0.1] = 0                      # empty leaves
    counts = rng.poisson(rng.uniform(0.5, 150), nl)
    counts[rng.random(nl) < 0.2] = 0                     # leaves no query visits
    wm.check([int(x) for x in sizes], [int(x) for x in counts], grid=256, qtile=qtile,
             chunk_tiles=int(rng.choice([8, 16, 20, 40])))


@pytest.mark.parametrize("sizes,counts", [
    ([5], [1]),                      # one pair
    ([0, 0, 40], [3, 1, 1]),         # empty leaves with queries
    ([0], [7]),                      # only an empty leaf
    ([700, 33, 0, 1], [0, 0, 0, 0]),  # no pairs at all
    ([4000] * 3, [200, 1, 64]),      # leaves of many chunks, full query tiles
])
def test_edge_shapes(sizes, counts):
    for qtile in (32, 64):
        wm.check(sizes, counts, grid=256, qtile=qtile)
