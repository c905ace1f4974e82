"""The scan's work list (tests/worklist_model.py restates the device code):
every scan workgroup's static share is covered by real work items, and every
tile of every (leaf, query tile) item is scanned exactly once, whatever the
leaf sizes and query counts (empty leaves, leaves without queries, a single
pair, totals smaller than the grid, leaves larger than a chunk)."""
import numpy as np
import pytest

import worklist_model as wm


@pytest.mark.parametrize("alpha", [0, 1, 7])
@pytest.mark.parametrize("small", [False, 2])
@pytest.mark.parametrize("seed", range(10))
def test_shares_cover_items_exactly_once(seed, small, alpha):
    rng = np.random.default_rng(seed)
    nl = int(rng.integers(1, 300))
    sizes = rng.integers(0, 3000, nl)
    sizes[rng.random(nl) < 0.1] = 0                      # empty leaves
    counts = rng.poisson(rng.uniform(0.5, 150), nl)
    counts[rng.random(nl) < 0.2] = 0                     # leaves no query visits
    wm.check([int(x) for x in sizes], [int(x) for x in counts], grid=int(rng.choice([64, 256, 3072])),
             chunk_tiles=int(rng.choice([8, 16, 20, 40])), small=small, alpha=alpha)


@pytest.mark.parametrize("sizes,counts", [
    ([5], [1]),                      # one pair
    ([0, 0, 40], [3, 1, 1]),         # empty leaves with queries
    ([0], [7]),                      # only an empty leaf
    ([700, 33, 0, 1], [0, 0, 0, 0]),  # no pairs at all
    ([4000] * 3, [200, 1, 64]),      # leaves of many chunks, full query tiles
])
def test_edge_shapes(sizes, counts):
    for small in (False, 2):
        for grid in (8, 256, 3072):
            for alpha in (0, 3, 40):
                wm.check(sizes, counts, grid=grid, small=small, alpha=alpha)


@pytest.mark.parametrize("seed", range(6))
def test_16_slot_tiles_only(seed):
    """Below 16 queries per leaf on average the work list holds 16-slot
    tiles only (kNarrowOnly): a leaf with c queries has ceil(c / 16) query
    tiles of weight 1, the pair of rank r sits in tile r // 16, slot r % 16,
    and a share may start inside any of them."""
    rng = np.random.default_rng(700 + seed)
    nl = int(rng.integers(50, 2000))
    sizes = rng.integers(0, 4000, nl)
    counts = rng.poisson(rng.uniform(1, 40), nl)
    wl = wm.check([int(x) for x in sizes], [int(x) for x in counts],
                  grid=int(rng.choice([256, 3072, 8192])), chunk_tiles=20, small=2)
    per_leaf = {}
    for leaf, n, j0, j1, q, w in wl["work"]:
        assert w == 1
        per_leaf[leaf] = max(per_leaf.get(leaf, 0), q + 1)
    for leaf, qt in per_leaf.items():
        assert qt == (int(counts[leaf]) + 15) // 16
    assert wm.query_tiles(17, 2) == (0, 2) and wm.query_tiles(16, 2) == (0, 1)
    assert wm.query_tiles(0, 2) == (0, 0) and wm.query_tiles(64, 2) == (0, 4)


@pytest.mark.parametrize("chunk_tiles", [8, 16])
@pytest.mark.parametrize("seed", range(4))
def test_item_capacity_at_small_chunks(seed, chunk_tiles):
    """The item buffer (MaxItems) holds every list at the smallest chunk
    smx_set_tuning accepts, in the 16-slot-only mode (ceil(c / 16) query
    tiles per leaf): e.g. 48 queries on every 64-tile leaf needs 3 x 8 = 24
    items per leaf, more than the 22.5 per leaf a pairs / 32 bound gave."""
    rng = np.random.default_rng(900 + seed)
    nl = int(rng.integers(20, 400))
    sizes = [64 * 32] * nl if seed == 0 else [int(x) for x in rng.integers(0, 4000, nl)]
    counts = [48] * nl if seed == 0 else [int(x) for x in rng.poisson(rng.uniform(1, 60), nl)]
    for small in (False, 2):
        for alpha in (0, 10):
            wm.check(sizes, counts, grid=256, chunk_tiles=chunk_tiles, small=small, alpha=alpha)
    if seed == 0:
        wl = wm.build(sizes, counts, 256, 8, 2)
        assert len(wl["work"]) == 24 * nl
        # the old pairs / 32 bound, at the chunk count this list really has
        assert len(wl["work"]) > (sum(counts) / 32 + nl) * 8
