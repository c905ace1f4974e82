#!/bin/bash
# Kernel trace of one generated-config bench (run on the GPU box):
#   CFG=deep1b bash tools/prof_config.sh <outdir>
set -e
OUT=${1:-gpurun_out/profc}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 800 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/trace" -o run \
  -- python3 "$ROOT/bench.py" --config ${CFG:-deep1b} --no-cpu-baseline --no-sweep --steps 10 --warmup 2 \
  > "$ROOT/$OUT/bench.json" 2> "$ROOT/$OUT/bench.err"
# the per-dispatch trace of the build phase is far larger than gpurun's
# copy-back limit: keep the per-kernel statistics only
rm -f "$ROOT/$OUT/trace/run_kernel_trace.csv"
