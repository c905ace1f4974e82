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


@pytest.mark.parametrize("seed", range(8))
def test_position_items_equal_listed_items(seed):
    """The fused front end's scan derives items from the positions
    (ItemFromPositions): every workgroup's segments equal the ones it lists
    from the materialized work list, including positions without pairs and
    more than 64 positions per share step."""
    rng = np.random.default_rng(100 + seed)
    nl = int(rng.integers(1, 400))
    sizes = rng.integers(0, 2500, nl)
    sizes[rng.random(nl) < 0.1] = 0
    counts = rng.poisson(rng.uniform(0.2, 90), nl)
    counts[rng.random(nl) < 0.3] = 0
    grid = int(rng.choice([64, 256, 3072]))
    wl = wm.build([int(x) for x in sizes], [int(x) for x in counts], grid, 32,
                  int(rng.choice([8, 20, 40])))
    for b in range(grid):
        assert wm.list_segments_pos(wl, b) == wm.list_segments(wl, b), f"workgroup {b}"


@pytest.mark.parametrize("seed", range(8))
def test_share_start_equals_wave_start(seed):
    """ShareStart (each scan workgroup's own search over the positions' unit
    prefix) gives the share start WaveStarts writes, position included."""
    rng = np.random.default_rng(200 + seed)
    nl = int(rng.integers(1, 2049))
    sizes = rng.integers(0, 3000, nl)
    sizes[rng.random(nl) < 0.1] = 0
    counts = rng.poisson(rng.uniform(0.2, 90), nl)
    counts[rng.random(nl) < 0.3] = 0
    grid = int(rng.choice([64, 256, 3072]))
    wl = wm.build([int(x) for x in sizes], [int(x) for x in counts], grid, 32,
                  int(rng.choice([8, 20, 40])))
    units = []
    for d in wl["pos"]:
        units.append(((d["cnt"] + 31) // 32) * ((d["n"] + 31) // 32))
    pu = np.concatenate([[0], np.cumsum(units)]).astype(int).tolist()
    for b in range(grid):
        ws, p = wm.share_start(wl, b, grid, pu)
        assert ws == wl["wave_start"][b], f"workgroup {b}"
        if ws[2] > 0:
            assert p == wl["wave_pos"][b], f"workgroup {b} position"
