# Round-4 measurement pass (gpurun, repo root): smoke, the glove trace and PMC
# passes, the scan's HBM traffic from that FETCH_SIZE pass (profiles/
# scan_traffic.json on the box, copied back under gpurun_out/), then the glove
# and SIFT bench lines with cpu_baseline and the SIFT trace/PMC passes.
set -o pipefail
O=gpurun_out/${TAG:-r04f}
mkdir -p $O
step() { echo "[r04_final] $(date +%T) $*" >&2; }
step smoke && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 &&
step prof_glove && timeout -k 10 900 bash tools/profile_bench.sh $O/prof_glove &&
step traffic && python tools/pmc_traffic.py $O/prof_glove/pmc1/run_counter_collection.csv > $O/traffic.log &&
cp profiles/scan_traffic.json $O/scan_traffic.json &&
step glove && timeout -k 10 600 python bench.py > $O/bench_glove.json 2> $O/bench_glove.err &&
step sift && timeout -k 10 600 python bench.py --config sift > $O/bench_sift.json 2> $O/bench_sift.err &&
step prof_sift && BENCH_ARGS="--config sift" timeout -k 10 900 bash tools/profile_bench.sh $O/prof_sift &&
step done
