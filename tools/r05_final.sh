#!/bin/bash
# Round-5 final measurement pass (gpurun, repo root): smoke, the GPU suite,
# the glove and SIFT traces + PMC passes and their traffic records, then the
# glove and SIFT lines (CPU baselines included) carrying them.
set -o pipefail
O=gpurun_out/${TAG:-r05y}
mkdir -p $O
step() { echo "[r05_final] $(date +%T) $*" >&2; }
step smoke && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 &&
step tests && timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
step prof_glove && timeout -k 10 900 bash tools/profile_bench.sh $O/prof_glove &&
python tools/pmc_traffic.py $O/prof_glove/pmc1/run_counter_collection.csv glove > $O/traffic_glove.log &&
step prof_sift && BENCH_ARGS="--config sift" timeout -k 10 900 bash tools/profile_bench.sh $O/prof_sift &&
python tools/pmc_traffic.py $O/prof_sift/pmc1/run_counter_collection.csv sift > $O/traffic_sift.log &&
cp profiles/scan_traffic_glove.json profiles/scan_traffic_sift.json $O/ &&
python tools/trace_overlap.py $O/prof_glove/trace/run_kernel_trace.csv > $O/prof_glove/overlap.txt &&
python tools/trace_overlap.py $O/prof_sift/trace/run_kernel_trace.csv > $O/prof_sift/overlap.txt &&
rm -f $O/prof_glove/trace/run_kernel_trace.csv $O/prof_sift/trace/run_kernel_trace.csv &&
step glove && timeout -k 10 600 python bench.py > $O/bench_glove.json 2> $O/bench_glove.err &&
step sift && timeout -k 10 600 python bench.py --config sift > $O/bench_sift.json 2> $O/bench_sift.err &&
step done
