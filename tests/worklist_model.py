"""A host model of the scan's work list (test infrastructure).

Restates, in Python, what the device builds per call
(scann_amd/csrc/smx_kernels.hip): PositionWork / WorklistFusedBlock (each
leaf position's items and units, their exclusive prefixes, the 8 XCD
groups' unit boundaries), ItemsCore (the work items and every scan
workgroup's static share) and the scan's ListSegments walk over a share.
`check()` asserts the invariants the scan relies on: every share's units are
covered by real items, the shares tile each group exactly, and every tile of
every (leaf, query tile) is scanned exactly once.
"""
from __future__ import annotations

import numpy as np

GROUPS = 8
ITEM_COST = 4   # smx_kernels.hip kItemCost


def chunks_of(n, chunk_tiles):
    tiles = (n + 31) // 32
    return 1 if tiles == 0 else (tiles + chunk_tiles - 1) // chunk_tiles


def chunk_tiles_range(n, chunk_tiles, ch):
    tiles = (n + 31) // 32
    chunks = 1 if tiles == 0 else (tiles + chunk_tiles - 1) // chunk_tiles
    return (tiles * ch) // chunks, (tiles * (ch + 1)) // chunks


def leaf_order(sizes):
    """smx_searcher.hip UploadIndex: descending size, dealt to the groups in
    a snake, each group contiguous."""
    nl = len(sizes)
    by_size = sorted(range(nl), key=lambda l: -sizes[l])   # stable
    order = []
    for g in range(GROUPS):
        for p in range(nl):
            r, i = divmod(p, GROUPS)
            if (i if r % 2 == 0 else GROUPS - 1 - i) == g:
                order.append(by_size[p])
    return order


def query_tiles(c, small=False):
    """(32-slot, 16-slot) query tiles of a leaf with c queries (LeafQueryTiles):
    small == 2 (kNarrowOnly): every query tile has 16 slots; otherwise every
    query tile has 32."""
    if small == 2:
        return 0, (c + 15) // 16
    return (c + 31) // 32, 0


def build(sizes, counts, grid, chunk_tiles, small=False, alpha=ITEM_COST):
    """Items (leaf, n, j0, jend, query tile, weight) and the workgroups'
    shares (first item, first tile, units).  A unit is a 16-slot tile: a
    32-slot item's tiles weigh 2, a 16-slot item's 1, and every item adds
    `alpha` units ahead of its first tile (kItemCost: its setup); a tile
    belongs to the share holding its first unit."""
    nl = len(sizes)
    order = leaf_order(sizes)
    items_p, units_p = [], []
    for p in range(nl):
        leaf = order[p]
        c, n = counts[leaf], sizes[leaf]
        q32, q16 = query_tiles(c, small)
        items_p.append((q32 + q16) * chunks_of(n, chunk_tiles))
        units_p.append((2 * q32 + q16) * ((n + 31) // 32) + alpha * items_p[-1])
    ex_i = np.concatenate([[0], np.cumsum(items_p)[:-1]]).astype(int)
    ex_u = np.concatenate([[0], np.cumsum(units_p)[:-1]]).astype(int)
    total_w = int(sum(units_p))
    wdiv = max(1, total_w)

    def group_of(x):
        return min(GROUPS - 1, (GROUPS * x) // wdiv)

    gunits = [None] * (GROUPS + 1)
    for p in range(nl):
        eu = int(ex_u[p])
        gp = group_of(eu)
        prev = group_of(eu - units_p[p - 1]) if p > 0 else -1
        for gg in range(prev + 1, gp + 1):
            gunits[gg] = eu
        if p == nl - 1:
            for gg in range(gp + 1, GROUPS + 1):
                gunits[gg] = total_w
    work = [None] * int(sum(items_p))
    slots = [None] * len(work)
    wave_start = [None] * grid
    for i in range(grid):
        g = i & (GROUPS - 1)
        if gunits[g + 1] == gunits[g]:
            wave_start[i] = (0, 0, 0)
    for p in range(nl):
        leaf = order[p]
        c, n = counts[leaf], sizes[leaf]
        chunks = chunks_of(n, chunk_tiles)
        q32, q16 = query_tiles(c, small)
        item0 = int(ex_i[p])
        for u in range((q32 + q16) * chunks):
            j0, j1 = chunk_tiles_range(n, chunk_tiles, u % chunks)
            q = u // chunks
            work[item0 + u] = (leaf, n, j0, j1, q, 2 if q < q32 else 1)
            # the query tile's leaf slots (ItemsCore: slot0 = leaf * stride +
            # first rank, nslots = min(width, c - first rank))
            r0 = 32 * q if q < q32 else 32 * q32 + 16 * (q - q32)
            width = 32 if q < q32 else 16
            slots[item0 + u] = (r0, min(width, c - r0))
        ua, ub = int(ex_u[p]), int(ex_u[p]) + units_p[p]
        if ua >= ub:
            continue
        g = group_of(ua)
        nw = (grid - g + GROUPS - 1) // GROUPS
        U0, span = gunits[g], gunits[g + 1] - gunits[g]
        k = ((ua - U0) * nw + span - 1) // span
        tiles = (n + 31) // 32
        while k < nw:
            us = U0 + (span * k) // nw
            if us >= ub:
                break
            ue = U0 + (span * (k + 1)) // nw
            off = us - ua
            # the query tile, then the chunk (item) holding unit `off`
            per32 = 2 * tiles + alpha * chunks
            if off < per32 * q32:
                q, r = divmod(off, per32)
                wt = 2
            else:
                q16i, r = divmod(off - per32 * q32, tiles + alpha * chunks)
                q, wt = q32 + q16i, 1
            ch = 0
            while True:
                a0, a1 = chunk_tiles_range(n, chunk_tiles, ch)
                if r < alpha + wt * (a1 - a0):
                    break
                r -= alpha + wt * (a1 - a0)
                ch += 1
            # the first tile whose first unit is >= off, and the units between
            if r <= alpha:
                j, skip = a0, alpha - r
            else:
                m = -(-(r - alpha) // wt)
                j, skip = a0 + m, wt * m - (r - alpha)
                if j == a1:                # the next item's first tile
                    skip += alpha
                    ch += 1
                    if ch == chunks:
                        q, ch = q + 1, 0
                    j = chunk_tiles_range(n, chunk_tiles, ch)[0] if q < q32 + q16 else 0
            wave_start[GROUPS * k + g] = (item0 + q * chunks + ch, j, max(0, ue - us - skip))
            k += 1
    return dict(order=order, work=work, slots=slots, wave_start=wave_start, gunits=gunits,
                total_w=total_w, chunk_tiles=chunk_tiles, alpha=alpha)


def list_segments(wl, b, max_segs=512):
    """The segments (item, j0, jend) of workgroup b's share, as ListSegments
    walks it (64 lanes per step): an item's tiles cost its weight in units;
    a partly taken item takes the tiles whose first unit is inside the share.
    Raises if a taken item is not a real one."""
    work = wl["work"]
    alpha = wl.get("alpha", 0)
    sw, sj, su = wl["wave_start"][b]
    first = True   # the share starts at a tile's first unit: no item cost
    segs = []
    while su > 0:
        used_lanes = 0
        excl = 0
        for lane in range(64):
            idx = sw + lane
            if excl >= su:
                break
            if idx >= len(work):
                raise AssertionError(f"share of workgroup {b} runs past the items (item {idx})")
            it = work[idx]
            w = it[5]
            f = first and lane == 0
            j0 = sj if f else it[2]
            ae = 0 if f else alpha
            t = max(0, it[3] - j0)
            used_lanes += 1
            take = min(t, -(-(su - excl - ae) // w)) if su - excl > ae else 0
            if take > 0:
                segs.append((idx, j0, j0 + take))
            excl += min(ae + t * w, su)
        sw += used_lanes
        su -= min(su, excl)
        sj, first = 0, False
    return segs


def max_items(sizes, pairs):
    """The workspace's item capacity (smx_searcher.hip MaxItems): (pairs / 16
    + nl + 1) x (ceil(max_tiles / 8) + 1)."""
    max_leaf = max(sizes) if len(sizes) else 0
    chunks = ((max_leaf + 31) // 32 + 7) // 8 + 1
    return (pairs // 16 + len(sizes) + 1) * chunks


def check(sizes, counts, grid=256, chunk_tiles=20, small=False, alpha=ITEM_COST):
    wl = build(sizes, counts, grid, chunk_tiles, small, alpha)
    cap = max_items(sizes, int(sum(counts)))
    assert len(wl["work"]) <= cap, f"{len(wl['work'])} items > MaxItems {cap}"
    assert all(w is not None for w in wl["wave_start"]), "a workgroup's share is not written"
    seen = {}
    for b in range(grid):
        for idx, j0, j1 in list_segments(wl, b):
            for t in range(j0, j1):
                key = (idx, t)
                assert key not in seen, f"tile {t} of item {idx} scanned twice"
                seen[key] = b
    # every tile of every item exactly once
    tiles = 0
    for idx, (leaf, n, j0, j1, qt, w) in enumerate(wl["work"]):
        for t in range(j0, j1):
            assert (idx, t) in seen, f"tile {t} of item {idx} (leaf {leaf}) never scanned"
        tiles += j1 - j0
    assert len(seen) == tiles
    # every chunk's query tiles cover the leaf's ranks 0..c-1 exactly once
    cover = {}
    for idx, (leaf, n, j0, j1, qt, w) in enumerate(wl["work"]):
        r0, ns = wl["slots"][idx]
        assert 0 < ns <= (32 if w == 2 else 16)
        cover.setdefault((leaf, j0), []).extend(range(r0, r0 + ns))
    for (leaf, j0), ranks in cover.items():
        assert sorted(ranks) == list(range(counts[leaf])), (leaf, j0)
    assert (sum((j1 - j0) * w for (_, _, j0, j1, _, w) in wl["work"])
            + alpha * len(wl["work"])) == wl["total_w"]
    return wl
