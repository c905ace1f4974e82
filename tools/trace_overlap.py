"""Overlap view of a rocprofv3 kernel trace of bench.py (batches in flight).

    python tools/trace_overlap.py <run_kernel_trace.csv> [first_scan] [count]

Takes `count` consecutive scan launches from the `first_scan`-th on (the
timed region), and for that window prints each pipeline kernel's launches,
mean duration, its share of the window, and how much of the window had 0, 1,
2, 3+ kernels running.
"""
import csv
import sys
from collections import defaultdict

import numpy as np


def short(name):
    for k in ("lut16_scan_kernel", "seed_tau_kernel", "final_select_rank_kernel",
              "topl_block_kernel", "partition_scores_kernel", "topl_sample_kernel",
              "final_select_kernel", "merge_shards_kernel"):
        if k in name:
            return k
    return name.split("(")[0][-40:]


def main(path, first=50, count=200):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                         r.get("Stream_Id", "")))
    rows.sort()
    scans = [r for r in rows if r[2] == "lut16_scan_kernel"]
    win = scans[first:first + count]
    t0, t1 = win[0][0], win[-1][1]
    sel = [r for r in rows if r[0] >= t0 and r[1] <= t1]
    per = defaultdict(list)
    for a, b, n, _ in sel:
        per[n].append(b - a)
    span = (t1 - t0) / 1e3
    print(f"window: {count} scans, {span:.1f} us = {span / count:.2f} us per batch")
    for n, d in sorted(per.items(), key=lambda x: -sum(x[1])):
        print(f"  {n:28s} n={len(d):4d} mean {np.mean(d) / 1e3:7.2f} us  sum/window {sum(d) / 1e3 / span:5.2f}")
    ev = []
    for a, b, n, _ in sel:
        ev.append((a, 1))
        ev.append((b, -1))
    ev.sort()
    hist = defaultdict(float)
    cur, last = 0, t0
    for t, d in ev:
        hist[min(cur, 3)] += t - last
        cur += d
        last = t
    tot = sum(hist.values())
    print("  concurrency: " + ", ".join(f"{k}{'+' if k == 3 else ''}: {v / tot:.2f}" for k, v in sorted(hist.items())))


if __name__ == "__main__":
    main(sys.argv[1], *(int(x) for x in sys.argv[2:4]))
