"""Print the smx kernels of a rocprofv3 --stats CSV (average microseconds per call).

    python tools/kstats_summary.py gpurun_out/kstats/run_kernel_stats.csv
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    name = r["Name"]
    if "smx" not in name and "rocclr" not in name:
        continue
    short = name.split("(")[0].replace("void ", "").replace("smx::(anonymous namespace)::", "")
    print(f"{short[:60]:60s} calls={int(r['Calls']):5d} avg_us={float(r['AverageNs']) / 1e3:9.2f} "
          f"total_ms={float(r['TotalDurationNs']) / 1e6:8.2f}")
