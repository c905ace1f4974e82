#!/bin/bash
# Round-5 pass: the -m gpu suite against the debug library (device bounds
# check on every computed index), the glove bench line, SIFT trace + PMC
# passes and its traffic record.
set -o pipefail
O=gpurun_out/${TAG:-r05g}
mkdir -p $O
step() { echo "[r05_g] $(date +%T) $*" >&2; }
step diag && SMX_LIB=scann_amd/lib/libscann_mi355x_diag.so timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/diag_tests.log 2>&1 &&
step glove && timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_glove.json 2> $O/bench_glove.err &&
step prof_sift && BENCH_ARGS="--config sift" timeout -k 10 900 bash tools/profile_bench.sh $O/prof_sift &&
step traffic && python tools/pmc_traffic.py $O/prof_sift/pmc1/run_counter_collection.csv sift > $O/traffic_sift.log &&
cp profiles/scan_traffic_sift.json $O/ &&
step done
