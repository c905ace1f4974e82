#!/bin/bash
# Kernel trace + stats of the bench per environment setting (GPU box, repo root):
#   ENVS="SMX_NARROW=1 SMX_NARROW=2" TAG=x BENCH_ARGS="--config deep1b" bash tools/trace_env.sh
# Output: gpurun_out/$TAG/<setting>/run_kernel_stats.csv (+ the trace, bench line)
set -o pipefail
ROOT=$(pwd)
O=$ROOT/gpurun_out/${TAG:-trace}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for E in ${ENVS:-SMX_NARROW=1}; do
  echo "[trace_env] $(date +%T) $E" >&2
  mkdir -p "$O/$E"
  (export ${E//,/ }; export SMX_LIB=${SMX_LIB:+$ROOT/$SMX_LIB}; timeout -k 10 ${LIMIT:-300} rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$O/$E" -o run -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-sweep --no-parity \
      --steps ${STEPS:-50} ${BENCH_ARGS:-} > "$O/$E/bench.json" 2> "$O/$E/bench.err") || exit 1
done
echo "[trace_env] done" >&2
