#!/bin/bash
# A/B of alternative builds of the library on one box: the bench line of each
# build (SMX_LIB=<lib>) for each configuration, interleaved REPS times.
#   LIBS="scann_amd/lib/libscann_mi355x.so scann_amd/lib/libscann_mi355x_x.so" \
#   CFGS="glove sift deep1b" REPS=2 TAG=x bash tools/ab_libs.sh
# Output: gpurun_out/$TAG/<config>.<lib>.json (one line per repetition).
# Builds: bash tools/build_rev.sh <rev> <name>, or hipcc with -D<knob> (the
# SMX_* compile knobs in scann_amd/csrc/smx_kernels.hip).
set -o pipefail
O=gpurun_out/${TAG:-abl}
mkdir -p $O
step() { echo "[ab_libs] $(date +%T) $*" >&2; }
for rep in $(seq ${REPS:-2}); do
  for L in ${LIBS:-scann_amd/lib/libscann_mi355x.so}; do
    n=$(basename $L .so)
    for C in ${CFGS:-glove}; do
      step "$C $n rep $rep" &&
      SMX_LIB=$L timeout -k 10 ${LIMIT:-400} python3 bench.py --config $C --steps ${STEPS:-200} --warmup 20 \
          --no-cpu-baseline --no-sweep --no-parity ${BENCH_ARGS:-} >> $O/$C.$n.json 2>> $O/bench.err || exit 1
    done
  done
done
step done
