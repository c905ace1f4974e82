#!/bin/bash
# configs[4] (16-slot tiles only) scan A/B on one box: the product library,
# alternative builds ($LIBS) and the timing library's ablations of the
# 16-slot kernel (SMX_SCAN_VARIANT: 4 no epilogue, 64 operands from the code
# registers instead of the LDS tables, 68 both; results invalid for those).
set -o pipefail
O=gpurun_out/${TAG:-r05n}
mkdir -p $O
CFG=${CFG:-deep1b}
A="--config $CFG --steps 60 --warmup 10 --no-cpu-baseline --no-sweep --no-parity"
step() { echo "[r05_narrow_ab] $(date +%T) $*" >&2; }
for rep in $(seq ${REPS:-1}); do
  for L in scann_amd/lib/libscann_mi355x.so ${LIBS:-}; do
    n=$(basename $L .so)
    step "$n rep $rep" && SMX_LIB=$L timeout -k 10 400 python3 bench.py $A >> $O/$CFG.$n.json 2>> $O/bench.err || exit 1
  done
done
for V in ${VARIANTS:-0 4 64 68}; do
  step "variant $V" && SMX_LIB=scann_amd/lib/libscann_mi355x_time.so SMX_SCAN_VARIANT=$V timeout -k 10 400 python3 bench.py $A >> $O/$CFG.time_v$V.json 2>> $O/bench.err || exit 1
done
step done
