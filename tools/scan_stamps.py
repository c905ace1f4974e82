"""Per-segment timeline of the LUT16 scan kernel (diagnostic variant 8).

    python tools/scan_stamps.py [chunk_tiles]      (on the GPU box)

Runs the glove-shaped bench search with scan variant 8, which writes one
record per work item (and one per wave start) to a separate buffer; the
library dumps the last call's records to $SMX_STAMPS.  Prints where a wave's
time goes: item setup (dependent loads, B fragments, sum limits), tiles,
flush (per-query atomics + copy), dequeue gaps, and the spread of wave start
and end times.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# the scan variants other than 0 exist only in the diagnostic library
os.environ.setdefault("SMX_LIB", os.path.join(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))), "scann_amd", "lib", "libscann_mi355x_time.so"))
import torch  # noqa: E402

from bench import LEAVES_TO_SEARCH, NQ, PRE_NN, FINAL_NN, build_index  # noqa: E402
from scann_amd import _native  # noqa: E402

WAVES = 12   # scan waves per workgroup (K <= 25)


def main():
    chunk = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    path = "/tmp/smx_stamps.bin"
    os.environ["SMX_STAMPS"] = path
    db, q, ix = build_index(1_183_514, seed=2)
    nat = _native.NativeIndex(ix)
    qd = torch.from_numpy(q).cuda()
    oi = torch.zeros((NQ, FINAL_NN), dtype=torch.int32, device="cuda")
    od = torch.zeros((NQ, FINAL_NN), dtype=torch.float32, device="cuda")
    nat.set_tuning(4096, 4, 8, chunk)
    for _ in range(4):
        nat.search_batched_device(qd.data_ptr(), NQ, LEAVES_TO_SEARCH, PRE_NN, FINAL_NN, True,
                                  oi.data_ptr(), od.data_ptr(), None)
    torch.cuda.synchronize()
    r = np.fromfile(path, dtype=np.uint64).reshape(-1, 8).astype(np.int64)
    blk = r[:, 0] >> 32
    xcc = r[:, 1] >> 32
    item = r[:, 1] & 0xFFFFFFFF
    rt, t0, t1, t2, t3 = r[:, 2], r[:, 3], r[:, 4], r[:, 5], r[:, 6]
    tiles, hits, surv = r[:, 7] & 0xFFFF, (r[:, 7] >> 16) & 0xFFFFFF, r[:, 7] >> 40
    start = item == 0xFFFFFFFF
    it = ~start
    print(f"records {len(r)}: wave starts {start.sum()}, items {it.sum()}, chunk {chunk}")
    # shader clock from items: memtime cycles per realtime tick (100 MHz)
    rt0 = rt.min()
    # wave start spread (realtime, us)
    ws = (rt[it] - rt0) / 100.0
    print(f"item start (us): min {ws.min():.2f} p50 {np.median(ws):.2f} p90 {np.percentile(ws, 90):.2f} max {ws.max():.2f}")
    # per item durations in shader cycles
    setup = t1[it] - t0[it]
    tl = t2[it] - t1[it]
    fl = t3[it] - t2[it]
    nt = tiles[it]
    print(f"item setup cycles: p50 {np.median(setup):.0f} p90 {np.percentile(setup, 90):.0f} mean {setup.mean():.0f}")
    per_tile = tl[nt > 0] / nt[nt > 0]
    print(f"tile cycles per tile: p50 {np.median(per_tile):.0f} p90 {np.percentile(per_tile, 90):.0f} mean {per_tile.mean():.0f}")
    print(f"flush cycles: p50 {np.median(fl):.0f} p90 {np.percentile(fl, 90):.0f} mean {fl.mean():.0f}")
    print(f"tiles per item: mean {nt.mean():.1f} max {nt.max()}")
    ht = hits[it][nt > 0] / nt[nt > 0]
    print(f"hit lanes per tile: mean {ht.mean():.2f} p50 {np.median(ht):.2f} p90 {np.percentile(ht, 90):.2f}; "
          f"survivors per item: mean {surv[it].mean():.1f} total {surv[it].sum()}; "
          f"hit lanes total {hits[it].sum()} (x16 sums tested)")
    # tile time vs hits
    hi = ht > np.percentile(ht, 75)
    print(f"tile cycles, items with hit rate above p75: {np.median(per_tile[hi]):.0f}, below: {np.median(per_tile[~hi]):.0f}")
    # per wave: items, end time, gaps
    order = np.lexsort((rt, blk))
    b_sorted, rt_s, t0_s, t3_s, it_s = blk[order], rt[order], t0[order], t3[order], it[order]
    ends, nitems, gaps, busy = [], [], [], []
    for b in np.unique(blk):
        m = b_sorted == b
        rts, t0b, t3b, itb = rt_s[m], t0_s[m], t3_s[m], it_s[m]
        items_b = itb.sum()
        nitems.append(items_b)
        # end = realtime of the last item's start + its duration in realtime
        # (clock from the wave's own first..last item)
        if items_b >= 1:
            ii = np.where(itb)[0]
            clk = None
            if len(ii) >= 2 and rts[ii[-1]] > rts[ii[0]]:
                clk = (t0b[ii[-1]] - t0b[ii[0]]) / ((rts[ii[-1]] - rts[ii[0]]) / 100.0)  # cycles/us
            dur_last = (t3b[ii[-1]] - t0b[ii[-1]]) / (clk or 2100.0)
            ends.append((rts[ii[-1]] - rt0) / 100.0 + dur_last)
            for a_, b_ in zip(ii[:-1], ii[1:]):
                gaps.append(t0b[b_] - t3b[a_])
            busy.append((t3b[ii] - t0b[ii]).sum() / (clk or 2100.0))
    ends = np.array(ends)
    nitems = np.array(nitems)
    print(f"items per wave: mean {nitems.mean():.2f} min {nitems.min()} max {nitems.max()}  waves {len(nitems)}")
    print(f"wave end (us): min {ends.min():.2f} p10 {np.percentile(ends, 10):.2f} p50 {np.median(ends):.2f} "
          f"p90 {np.percentile(ends, 90):.2f} max {ends.max():.2f}")
    if gaps:
        gaps = np.array(gaps)
        print(f"dequeue gap cycles: p50 {np.median(gaps):.0f} p90 {np.percentile(gaps, 90):.0f}")
    busy = np.array(busy)
    print(f"wave busy (us): p50 {np.median(busy):.2f} mean {busy.mean():.2f}")
    # per wave: first item start, per SIMD: waves and tiles
    hw = r[:, 0] & 0xFFFFFFFF
    first = {}
    last_end = {}
    for i in np.where(it)[0]:
        b = blk[i]
        st_us = (rt[i] - rt0) / 100.0
        first[b] = min(first.get(b, 1e18), st_us)
    fs = np.array(list(first.values()))
    print(f"wave first-item start (us): min {fs.min():.2f} p50 {np.median(fs):.2f} p90 {np.percentile(fs, 90):.2f} max {fs.max():.2f}")
    simd = (xcc << 16) | ((hw >> 8) & 0xFFF) << 2 | ((hw >> 4) & 3)
    waves_per_simd = {}
    tiles_per_simd = {}
    for i in np.where(it)[0]:
        k = int(simd[i])
        waves_per_simd.setdefault(k, set()).add(int(blk[i]))
        tiles_per_simd[k] = tiles_per_simd.get(k, 0) + int(tiles[i])
    wps = np.array([len(v) for v in waves_per_simd.values()])
    tps = np.array(list(tiles_per_simd.values()))
    print(f"SIMDs {len(wps)}: waves/SIMD min {wps.min()} p50 {np.median(wps):.0f} max {wps.max()}; "
          f"tiles/SIMD min {tps.min()} p50 {np.median(tps):.0f} max {tps.max()}")
    cu = (xcc << 16) | ((hw >> 8) & 0xFFF)
    u, cnts = np.unique(cu[it], return_counts=True)
    wpc = {}
    for i in np.where(it)[0]:
        wpc.setdefault(int(cu[i]), set()).add(int(blk[i]))
    wpcv = np.array([len(v) for v in wpc.values()])
    print(f"CUs {len(wpcv)}: waves/CU min {wpcv.min()} p50 {np.median(wpcv):.0f} max {wpcv.max()}")
    # per group: wave ends and busy
    wend = {}
    for b in np.unique(blk):
        m = (blk == b) & it
        ii = np.where(m)[0]
        j = ii[np.argmax(rt[ii])]
        wend[int(b)] = (rt[j] - rt0) / 100.0 + (t3[j] - t0[j]) / 2100.0
    grp = (blk // WAVES) % 8   # worker = workgroup * WAVES + wave; workgroup % 8 = XCD group
    for gsel in range(8):
        e = np.array([v for k, v in wend.items() if (k // WAVES) % 8 == gsel])
        hm = hits[(grp == gsel) & it].sum()
        print(f"group {gsel}: wave end p10 {np.percentile(e, 10):.1f} p50 {np.median(e):.1f} max {e.max():.1f} us; hits {hm}")
    # per SIMD: end vs hits
    send, shits = {}, {}
    for i in np.where(it)[0]:
        k = int(simd[i])
        send[k] = max(send.get(k, 0.0), wend[int(blk[i])])
        shits[k] = shits.get(k, 0) + int(hits[i])
    ks = list(send)
    e = np.array([send[k] for k in ks]); hh = np.array([shits[k] for k in ks])
    print(f"SIMD end: p10 {np.percentile(e, 10):.1f} p50 {np.median(e):.1f} p90 {np.percentile(e, 90):.1f} max {e.max():.1f}; "
          f"corr(end, hits) {np.corrcoef(e, hh)[0, 1]:.2f}")
    # per workgroup (CU share): end time vs its hits, segments (setups), tiles
    wg = blk // WAVES
    wgs = np.unique(wg[it])
    wend_g, whits_g, wseg_g, wtil_g = [], [], [], []
    for g_ in wgs:
        m = (wg == g_) & it
        ii = np.where(m)[0]
        wend_g.append(max(wend[int(b)] for b in np.unique(blk[ii])))
        whits_g.append(hits[ii].sum())
        wseg_g.append(len(ii))
        wtil_g.append(tiles[ii].sum())
    wend_g, whits_g, wseg_g, wtil_g = map(np.array, (wend_g, whits_g, wseg_g, wtil_g))
    print(f"workgroups {len(wgs)}: end p10 {np.percentile(wend_g, 10):.1f} p50 {np.median(wend_g):.1f} "
          f"p90 {np.percentile(wend_g, 90):.1f} max {wend_g.max():.1f}; tiles min {wtil_g.min()} max {wtil_g.max()}; "
          f"segments p50 {np.median(wseg_g):.0f} max {wseg_g.max()}")
    for nm, v in (("hits", whits_g), ("segments", wseg_g), ("tiles", wtil_g)):
        print(f"    corr(end, {nm}) {np.corrcoef(wend_g, v)[0, 1]:.2f}")
    slow = np.argsort(wend_g)[-5:]
    for i in slow:
        print(f"    slow wg {wgs[i]}: end {wend_g[i]:.1f} hits {whits_g[i]} segments {wseg_g[i]} tiles {wtil_g[i]}")
    # XCC placement of the groups
    for gsel in range(8):
        m = (grp == gsel) & it
        if m.any():
            u, c = np.unique(xcc[m], return_counts=True)
            print(f"group {gsel}: xcc {dict(zip(u.tolist(), c.tolist()))}")


if __name__ == "__main__":
    main()
