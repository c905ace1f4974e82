"""Summarise bench JSON lines: value, ms/step, scan launch, stage times."""
import json
import sys

for f in sys.argv[1:]:
    print("==", f)
    for line in open(f):
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        r = d.get("roofline", {})
        st = {k.replace("_ms", ""): round(v * 1000, 1) for k, v in d.get("stage_ms", {}).items()}
        print(f"  {d['value']:.4g} {d['ms_per_step']} scan {r.get('avg_launch_ms')} "
              f"frac {r.get('frac')} useful {r.get('useful_mfma_frac')} "
              f"recall {d.get('recall_at_10')} cand_max {d.get('candidates_max')} {st}")
