"""Average per-launch PMC values (skipping warm-up launches) of pmc_scan.sh output dirs.

    python tools/pmc_summary.py gpurun_out/pmc_v0 gpurun_out/pmc_v8
"""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    acc = collections.defaultdict(list)
    for f in sorted(glob.glob(d + "/p*/run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(d)
    for k, v in sorted(acc.items()):
        v = v[2:] or v
        print(f"  {k:32s} {sum(v) / len(v) / 1e6:12.3f} M")
