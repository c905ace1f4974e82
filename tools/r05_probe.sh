#!/bin/bash
# Round-5 probes (gpurun, repo root): two batches in flight (overlap_probe),
# the seed at 2048 rows (SMX_SEED_PER_THREAD=8 build) vs 4096, and the
# front-end / select phase stamps.
set -o pipefail
O=gpurun_out/${TAG:-r05c}
mkdir -p $O
step() { echo "[r05_probe] $(date +%T) $*" >&2; }
step overlap && timeout -k 10 300 python3 tools/overlap_probe.py --steps 300 > $O/overlap.log 2>&1 &&
step seed8 && TAG=$(basename $O)/ab LIBS="scann_amd/lib/libscann_mi355x.so scann_amd/lib/libscann_mi355x_seed8.so" STEPS=300 bash tools/ab_libs.sh &&
step phases && timeout -k 10 300 python3 tools/phase_stamps.py 4 > $O/phases.log 2>&1 &&
step done
