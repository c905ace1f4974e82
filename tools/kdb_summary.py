"""Per-kernel average durations from a rocprofv3 --kernel-trace database
(rocpd SQLite, the default output format of ROCm 7.2's rocprofv3).

    python tools/kdb_summary.py gpurun_out/x/trace/run_results.db
"""
import re
import sqlite3
import sys
from collections import defaultdict

db = sqlite3.connect(sys.argv[1])
rows = db.execute(
    "select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d "
    "join rocpd_info_kernel_symbol s on d.kernel_id = s.id").fetchall()
acc = defaultdict(list)
for name, t0, t1 in rows:
    short = re.sub(r"^void ", "", name).replace("smx::(anonymous namespace)::", "")
    short = re.sub(r"\((smx::|float|int|unsigned|const|HIP).*$", "", short)
    acc[short].append((t1 - t0) / 1e3)
for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
    v.sort()
    print(f"{k[:56]:56s} calls={len(v):5d} avg_us={sum(v) / len(v):8.2f} "
          f"p50_us={v[len(v) // 2]:8.2f} total_ms={sum(v) / 1e3:8.2f}")
