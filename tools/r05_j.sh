#!/bin/bash
# A/B of the work-item chunk and the seed leaves with three batches in flight
set -o pipefail
O=gpurun_out/${TAG:-r05j}
mkdir -p $O
step() { echo "[r05_j] $(date +%T) $*" >&2; }
step chunk && TAG=$(basename $O)/chunk ENVS="SMX_CHUNK_TILES=12 SMX_CHUNK_TILES=16 SMX_CHUNK_TILES=20 SMX_CHUNK_TILES=28" STEPS=300 BENCH_ARGS="--no-latency" bash tools/ab_env.sh &&
step seed && TAG=$(basename $O)/seed ENVS="SMX_SEED_LEAVES=2 SMX_SEED_LEAVES=3 SMX_SEED_LEAVES=4 SMX_SEED_LEAVES=6" STEPS=300 BENCH_ARGS="--no-latency" bash tools/ab_env.sh &&
step done
