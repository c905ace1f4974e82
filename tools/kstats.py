"""Per-kernel average durations of rocprofv3 --stats runs (smx kernels called
at least 100 times) and the bench line next to each: tools/trace_env.sh output.

    python tools/kstats.py gpurun_out/<tag>/*/
"""
import csv
import os
import subprocess
import sys

for d in sys.argv[1:]:
    print("==", d)
    tot = 0.0
    for x in csv.DictReader(open(os.path.join(d, "run_kernel_stats.csv"))):
        if "smx" in x["Name"] and int(x["Calls"]) >= 100 and "nearest" not in x["Name"]:
            us = float(x["AverageNs"]) / 1000
            tot += us
            print("  %-66s %6s %8.1f us" % (x["Name"][:66], x["Calls"], us))
    print("  sum %.1f" % tot)
    b = os.path.join(d, "bench.json")
    if os.path.exists(b):
        subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "abs.py"), b])
