"""Print the smx kernels of a rocprofv3 --stats CSV (average microseconds per call).

    python tools/kstats_summary.py gpurun_out/prof/trace/run_kernel_stats.csv
"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    name = r["Name"]
    if "smx" not in name and "rocclr" not in name:
        continue
    short = re.sub(r"^void ", "", name)
    short = short.replace("smx::(anonymous namespace)::", "")
    short = re.sub(r"\((smx::|float|int|unsigned|const|HIP).*$", "", short)
    print(f"{short[:48]:48s} calls={int(r['Calls']):5d} avg_us={float(r['AverageNs']) / 1e3:9.2f} "
          f"total_ms={float(r['TotalDurationNs']) / 1e6:8.2f}")
