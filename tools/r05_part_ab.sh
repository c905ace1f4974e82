#!/bin/bash
# Multi-tile partition kernel: the GPU suite, then same-box A/B of the
# product library against $BASE on the shard configurations and glove.
set -o pipefail
O=gpurun_out/${TAG:-r05pa}
mkdir -p $O
step() { echo "[r05_part_ab] $(date +%T) $*" >&2; }
step tests && timeout -k 10 500 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
for rep in 1 2; do
  for L in scann_amd/lib/libscann_mi355x.so ${BASE:-scann_amd/lib/libscann_mi355x_base.so}; do
    n=$(basename $L .so)
    for C in deep1b soar100m; do
      step "$C $n rep $rep" && SMX_LIB=$L timeout -k 10 400 python3 bench.py --config $C --steps 60 --warmup 10 --no-cpu-baseline --no-sweep --no-parity >> $O/$C.$n.json 2>> $O/bench.err || exit 1
    done
  done
done
step done
