#!/bin/bash
# A/B of environment switches of the product library on one box: the bench
# line of each setting, interleaved twice.
#   ENVS="SMX_NARROW=0 SMX_NARROW=1,SMX_LUT_SPLIT=0" TAG=x STEPS=200 BENCH_ARGS="--config deep1b" bash tools/ab_env.sh
# A setting is one or more VAR=value joined by commas.
# Output: gpurun_out/$TAG/<setting>.json (one line per repetition).
set -o pipefail
O=gpurun_out/${TAG:-abe}
mkdir -p $O
step() { echo "[ab_env] $(date +%T) $*" >&2; }
for rep in 1 2; do
  for E in ${ENVS:-SMX_NARROW=1}; do
    step "$E rep $rep" &&
    env ${E//,/ } timeout -k 10 ${LIMIT:-240} python3 bench.py --steps ${STEPS:-200} --warmup 10 \
        --no-cpu-baseline --no-sweep ${BENCH_ARGS:-} >> $O/$E.json 2>> $O/bench.err || exit 1
  done
done
step done
