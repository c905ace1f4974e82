#!/bin/bash
# One batch at a time under rocprofv3 (GPU box, repo root): every scan launch
# runs alone on the device (one stream: the per-batch kernels serialise), so
# the kernel-trace average of the scan is the duration the bench line's
# roofline.frac divides by (HIP events around the scan, replayed alone).
#   [BENCH_ARGS="--config sift"] bash tools/profile_alone.sh <outdir>
# then: python tools/roofline_check.py <outdir>
set -e
OUT=${1:-gpurun_out/prof_alone}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/trace" -o run \
  -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-sweep --no-parity --in-flight 1 --steps 50 \
  ${BENCH_ARGS:-} > "$ROOT/$OUT/bench.json" 2> "$ROOT/$OUT/bench.err"
cd "$ROOT"
python tools/kstats_summary.py "$OUT/trace/run_kernel_stats.csv" > "$OUT/kernel_summary.txt"
cp "$OUT/trace/run_kernel_stats.csv" "$OUT/kernel_stats.csv"
rm -f "$OUT"/trace/run_kernel_trace.csv
