#!/bin/bash
# Seed row budget A/B (GPU box, repo root): the glove line at leaves_to_search
# 20 and 100 for each SMX_SEED_ROWS, one box:
#   ROWS="1024 2048 4096" LS="20 100" [STEPS=200 WARMUP=20 REPS=1] bash tools/seed_rows_ab.sh <outdir>
set -o pipefail
O=${1:-gpurun_out/seed_rows}
mkdir -p $O
for rep in $(seq 1 ${REPS:-1}); do
for L in ${LS:-20 100}; do
  for R in ${ROWS:-1024 2048 4096}; do
    SMX_SEED_ROWS=$R timeout -k 10 300 python bench.py --no-cpu-baseline --no-sweep \
      --steps ${STEPS:-200} --warmup ${WARMUP:-20} --leaves-to-search $L \
      > $O/L${L}_rows${R}_r${rep}.json 2> $O/L${L}_rows${R}_r${rep}.err || exit 1
  done
done
done
python - "$O" <<'PY'
import json, glob, sys
for f in sorted(glob.glob(sys.argv[1] + "/L*_rows*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    st = d["stage_ms"]
    print(f"{f.split('/')[-1]:22s} qps {d['value']/1e6:6.3f}M single {d['single_stream']['qps']/1e6:6.3f}M "
          f"seed {st['seed_scan_ms']*1e3:5.1f} scan {st['scan_ms']*1e3:5.1f} select {st['select_ms']*1e3:5.1f} "
          f"total {st['total_ms']*1e3:6.1f} cand {d['candidates_mean']:6.1f} recall {d['recall_at_10']} "
          f"mismatch {d['parity_vs_oracle']['id_mismatch']}")
PY
