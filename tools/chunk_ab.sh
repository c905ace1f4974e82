#!/bin/bash
# Work-item chunk (tiles per item) A/B on one box: the glove line per
# SMX_CHUNK_TILES value at leaves_to_search 100 and 15, REPS times.
#   CHUNKS="12 16 20 28 40" LS="100 15" REPS=2 bash tools/chunk_ab.sh <outdir>
set -o pipefail
O=${1:-gpurun_out/chunk_ab}
mkdir -p $O
for rep in $(seq 1 ${REPS:-2}); do
  for L in ${LS:-100 15}; do
    for C in ${CHUNKS:-12 16 20 28 40}; do
      SMX_CHUNK_TILES=$C timeout -k 10 300 python bench.py --no-cpu-baseline --no-sweep \
        --steps ${STEPS:-100} --warmup 20 --leaves-to-search $L \
        > $O/L${L}_chunk${C}_r${rep}.json 2> /dev/null || exit 1
    done
  done
done
python - "$O" <<'PY'
import json, glob, sys
for f in sorted(glob.glob(sys.argv[1] + "/L*_chunk*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    st = d["stage_ms"]
    print(f"{f.split('/')[-1]:24s} qps {d['value']/1e6:6.3f}M single {d['single_stream']['qps']/1e6:6.3f}M "
          f"scan {st['scan_ms']*1e3:5.1f} total {st['total_ms']*1e3:6.1f}")
PY
