#!/bin/bash
# A/Bs: the v_perm hit packing (product vs base library, glove, in flight and
# alone); SIFT (new data) 16-slot-only vs 32-slot tiles.
set -o pipefail
O=gpurun_out/${TAG:-r05i}
mkdir -p $O
step() { echo "[r05_i] $(date +%T) $*" >&2; }
step libs && TAG=$(basename $O)/libs LIBS="scann_amd/lib/libscann_mi355x_base.so scann_amd/lib/libscann_mi355x.so" STEPS=300 BENCH_ARGS="--no-parity" bash tools/ab_libs.sh &&
step sift_narrow && TAG=$(basename $O)/sift_narrow ENVS="SMX_NARROW=0 SMX_NARROW=2" STEPS=300 BENCH_ARGS="--config sift --in-flight 1 --no-latency" bash tools/ab_env.sh &&
step done
