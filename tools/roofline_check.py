"""The bench line's kernel-alone roofline recomputed from the kept rocprofv3
summary of the same command (tools/profile_alone.sh):

    python tools/roofline_check.py profiles/r06/prof_glove_alone

frac = algorithmic int8 ops per launch (64 per code byte) / the
rocprof average duration of the scan kernel / the smfmac peak; printed beside
the line's own frac (HIP events) and their ratio.
"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import HBM_PEAK_BPS, SMFMAC_PEAK_TOPS  # noqa: E402

d = sys.argv[1]
line = json.loads(open(os.path.join(d, "bench.json")).read().strip().splitlines()[-1])
roof = line["roofline"]
rows = [r for r in csv.DictReader(open(os.path.join(d, "kernel_stats.csv")))
        if "lut16_scan_kernel" in r["Name"]]
calls = sum(int(r["Calls"]) for r in rows)
avg_ns = sum(float(r["TotalDurationNs"]) for r in rows) / calls
ops = float(roof["algorithmic_ops_per_launch"])
frac = ops / (avg_ns * 1e-9) / 1e12 / SMFMAC_PEAK_TOPS
out = {"scan_kernel": [r["Name"][:80] for r in rows], "rocprof_calls": calls,
       "rocprof_avg_us": round(avg_ns / 1e3, 2), "rocprof_frac": round(frac, 4),
       "line_avg_us": round(roof["avg_launch_ms"] * 1e3, 2), "line_frac": roof["frac"],
       "ratio": round(frac / roof["frac"], 4), "ms_per_step": line["ms_per_step"]}
if roof.get("traffic"):
    out["rocprof_hbm_frac"] = round(roof["traffic"] / (avg_ns * 1e-9) / HBM_PEAK_BPS, 4)
print(json.dumps(out, indent=1))
