#!/bin/bash
# A/B of the front end on one box: fused (topl+seed, worklist+scatter) vs the
# separate launches, kernel trace of each, then the plain bench lines.
set -o pipefail
O=gpurun_out/${TAG:-ab}
mkdir -p $O
step() { echo "[ab] $(date +%T) $*" >&2; }
export TMPDIR=/tmp
for F in 1 0; do
  step "trace fused=$F" &&
  SMX_FUSED_FRONT=$F timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/trace$F -o run -- \
      python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-sweep > $O/trace$F.log 2>&1 || exit 1
done
for F in 1 0 1 0; do
  step "bench fused=$F" &&
  SMX_FUSED_FRONT=$F timeout -k 10 240 python3 bench.py --steps 200 --warmup 10 --no-cpu-baseline \
      --no-sweep >> $O/bench$F.json 2>> $O/bench.err || exit 1
done
step done
