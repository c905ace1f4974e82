#!/bin/bash
# Round-5 final measurement pass (gpurun, repo root): smoke, the GPU suite,
# the glove line (CPU baseline included), its trace + PMC passes and traffic
# record, the SIFT line with its CPU baseline.
set -o pipefail
O=gpurun_out/${TAG:-r05z}
mkdir -p $O
step() { echo "[r05_final] $(date +%T) $*" >&2; }
step smoke && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 &&
step tests && timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
step prof_glove && timeout -k 10 900 bash tools/profile_bench.sh $O/prof_glove &&
step traffic && python tools/pmc_traffic.py $O/prof_glove/pmc1/run_counter_collection.csv glove > $O/traffic.log &&
cp profiles/scan_traffic_glove.json $O/scan_traffic_glove.json &&
step glove && timeout -k 10 600 python bench.py > $O/bench_glove.json 2> $O/bench_glove.err &&
step sift && timeout -k 10 600 python bench.py --config sift > $O/bench_sift.json 2> $O/bench_sift.err &&
step done
