#!/bin/bash
# Round-5 check of the pair-record pipeline: GPU suite, bench at 1/2/3
# batches in flight, the 16-slot mixed mode at glove's recall gate (L = 20),
# a kernel trace of the default bench.
set -o pipefail
O=gpurun_out/${TAG:-r05e}
mkdir -p $O
step() { echo "[r05_e] $(date +%T) $*" >&2; }
step tests && timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 &&
for f in 1 2 3; do
  step "bench in-flight $f" && timeout -k 10 200 python bench.py --in-flight $f --no-cpu-baseline --no-sweep --steps 300 >> $O/bench_fl.json 2>> $O/bench.err || exit 1
done &&
step narrow && TAG=$(basename $O)/narrow ENVS="SMX_NARROW=0 SMX_NARROW=1 SMX_NARROW=2" STEPS=300 BENCH_ARGS="--leaves-to-search 20 --in-flight 1" LIMIT=200 bash tools/ab_env.sh &&
step trace && R=$(pwd) && cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace -o run -- python3 $R/bench.py --no-cpu-baseline --no-sweep --no-parity --steps 100 > $R/$O/bench_traced.json 2> $R/$O/bench_traced.err &&
step done
