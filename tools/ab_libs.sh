#!/bin/bash
# A/B of alternative builds of the library on one box: the bench line of each
# (SMX_LIB=<lib>), interleaved twice.  LIBS="a.so b.so" (default: product).
set -o pipefail
O=gpurun_out/${TAG:-abl}
mkdir -p $O
step() { echo "[ab_libs] $(date +%T) $*" >&2; }
for rep in 1 2; do
  for L in ${LIBS:-scann_amd/lib/libscann_mi355x.so}; do
    n=$(basename $L .so)
    step "$n rep $rep" &&
    SMX_LIB=$L timeout -k 10 ${LIMIT:-240} python3 bench.py --steps ${STEPS:-200} --warmup 10 --no-cpu-baseline \
        --no-sweep ${BENCH_ARGS:-} >> $O/$n.json 2>> $O/bench.err || exit 1
  done
done
step done
