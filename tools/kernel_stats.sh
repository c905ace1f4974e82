#!/bin/bash
# Per-kernel durations of the glove-shaped search (rocprofv3 kernel trace).
#   bash tools/kernel_stats.sh <tune.py config> <outdir>     (on the GPU box)
set -e
CFG=${1:-4096,2,0,32}
OUT=${2:-gpurun_out/kstats}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT" -o run \
  -- python3 "$ROOT/tools/tune.py" "$CFG" > "$ROOT/$OUT/run.log" 2>&1
