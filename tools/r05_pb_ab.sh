#!/bin/bash
# Partition blocks target (SMX_PART_BLOCKS builds) A/B: sift, soar100m, deep1b.
set -o pipefail
O=gpurun_out/${TAG:-r05pb}
mkdir -p $O
step() { echo "[r05_pb_ab] $(date +%T) $*" >&2; }
for rep in 1 2; do
  for L in scann_amd/lib/libscann_mi355x.so $LIBS; do
    n=$(basename $L .so)
    for C in ${CFGS:-sift soar100m deep1b}; do
      step "$C $n rep $rep" && SMX_LIB=$L timeout -k 10 300 python3 bench.py --config $C --steps 100 --warmup 20 --no-cpu-baseline --no-sweep --no-parity >> $O/$C.$n.json 2>> $O/bench.err || exit 1
    done
  done
done
step done
