# Round-4 measurement pass (gpurun, repo root): smoke, glove and SIFT bench
# lines with cpu_baseline, their rocprofv3 kernel traces and PMC passes.
set -o pipefail
O=gpurun_out/${TAG:-r04f}
mkdir -p $O
step() { echo "[r04_final] $(date +%T) $*" >&2; }
step smoke && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 &&
step glove && timeout -k 10 600 python bench.py > $O/bench_glove.json 2> $O/bench_glove.err &&
step prof_glove && timeout -k 10 900 bash tools/profile_bench.sh $O/prof_glove &&
step sift && timeout -k 10 600 python bench.py --config sift > $O/bench_sift.json 2> $O/bench_sift.err &&
step prof_sift && BENCH_ARGS="--config sift" timeout -k 10 900 bash tools/profile_bench.sh $O/prof_sift &&
step done
