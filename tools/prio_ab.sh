#!/bin/bash
# A/B of per-stream priorities for the in-flight batches (bench.py's
# SMX_BENCH_STREAM_PRIORITY), at the driver's 20 steps and at 200, REPS times
# interleaved:  PRIOS="none -1,0,0 -1,-1,0" REPS=3 bash tools/prio_ab.sh <outdir>
set -o pipefail
O=$1; mkdir -p $O
for rep in $(seq ${REPS:-3}); do
  for P in ${PRIOS:-none -1,0,0}; do
    for S in 20 200; do
      if [ "$P" = none ]; then E=""; else E="$P"; fi
      SMX_BENCH_STREAM_PRIORITY="$E" timeout -k 10 300 python3 bench.py --steps $S --warmup 5 \
        --no-cpu-baseline --no-sweep --no-parity --no-latency >> $O/p${P}_s$S.json 2>> $O/err.log || exit 1
    done
  done
done
