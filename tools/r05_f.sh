#!/bin/bash
# Round-5 pass: GPU suite, glove and SIFT bench lines (no CPU baseline), the
# glove trace + PMC passes.
set -o pipefail
O=gpurun_out/${TAG:-r05f}
mkdir -p $O
step() { echo "[r05_f] $(date +%T) $*" >&2; }
step tests && timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 &&
step glove && timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_glove.json 2> $O/bench_glove.err &&
step sift && timeout -k 10 400 python bench.py --config sift --no-cpu-baseline > $O/bench_sift.json 2> $O/bench_sift.err &&
step prof_glove && timeout -k 10 900 bash tools/profile_bench.sh $O/prof_glove &&
step traffic && python tools/pmc_traffic.py $O/prof_glove/pmc1/run_counter_collection.csv glove > $O/traffic.log &&
cp profiles/scan_traffic_glove.json $O/ &&
step done
