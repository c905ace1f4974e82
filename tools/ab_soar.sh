#!/bin/bash
# A/B of library builds on the configs[3] shard bench (SMX_LIB=<lib>):
#   LIBS="a.so b.so" bash tools/ab_soar.sh   (output gpurun_out/$TAG/)
set -o pipefail
O=gpurun_out/${TAG:-abs}
mkdir -p $O
for rep in ${REPS:-1 2}; do
  for L in $LIBS; do
    n=$(basename $L .so)
    echo "[ab_soar] $(date +%T) $n rep $rep" >&2
    SMX_LIB=$L timeout -k 10 400 python3 bench.py --config ${CFG:-soar100m} --steps 30 --warmup 5 \
        --no-cpu-baseline --no-sweep >> $O/$n.json 2>> $O/bench.err || exit 1
  done
done
