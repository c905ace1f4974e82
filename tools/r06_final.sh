#!/bin/bash
# Round-6 final measurement pass (gpurun, repo root), in parts so each fits
# one call:  PART=a|b|c TAG=r06z bash tools/r06_final.sh
#  a: smoke, the GPU suite, the one-batch-at-a-time rocprof summaries of glove
#     and SIFT (tools/profile_alone.sh + roofline_check.py), the glove and
#     SIFT FETCH_SIZE passes (traffic records keyed by the kernel source);
#  b: the glove and SIFT lines (CPU baselines included), the glove line with
#     --scaling strong;
#  c: configs[3] / configs[4]: FETCH_SIZE passes, the deep1b alone profile,
#     both shard lines (parity, CPU baseline with the emulate mismatch).
set -o pipefail
O=gpurun_out/${TAG:-r06z}
ROOT=$(pwd)
mkdir -p $O
step() { echo "[r06_final] $(date +%T) $*" >&2; }
fetch() {   # <config>
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 500 rocprofv3 --pmc FETCH_SIZE --output-format csv \
    -d "$ROOT/$O/pmc_$1" -o run --kernel-include-regex "lut16_scan_kernel" -- python3 "$ROOT/bench.py" \
    --config $1 --no-cpu-baseline --no-sweep --no-parity --no-latency --steps 20 > "$ROOT/$O/pmc_$1.log" 2>&1) &&
  python tools/pmc_traffic.py $O/pmc_$1/run_counter_collection.csv $1 > $O/traffic_$1.log &&
  cp profiles/scan_traffic_$1.json $O/ && rm -rf $O/pmc_$1
}
alone() {   # <config>
  BENCH_ARGS="--config $1" timeout -k 10 900 bash tools/profile_alone.sh $O/prof_$1_alone &&
  python tools/roofline_check.py $O/prof_$1_alone > $O/prof_$1_alone/roofline_check.json
}
case ${PART:-a} in
a)
  step smoke && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 &&
  step tests && timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 900 --timeout-method thread --durations=10 > $O/gpu_tests.log 2>&1 &&
  step fetch_glove && fetch glove && step fetch_sift && fetch sift &&
  step alone_glove && alone glove && step alone_sift && alone sift &&
  step diag_tests && SMX_LIB=scann_amd/lib/libscann_mi355x_diag.so timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 900 --timeout-method thread > $O/diag_tests.log 2>&1 &&
  step done ;;
b)
  step glove && timeout -k 10 600 python bench.py > $O/bench_glove.json 2> $O/bench_glove.err &&
  step glove_s20 && timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_glove_s20.json 2> $O/bench_glove_s20.err &&
  step strong && timeout -k 10 600 python bench.py --no-cpu-baseline --scaling strong > $O/bench_glove_strong.json 2> $O/bench_glove_strong.err &&
  step sift && timeout -k 10 600 python bench.py --config sift > $O/bench_sift.json 2> $O/bench_sift.err && step done ;;
c)
  step fetch_soar && fetch soar100m && step fetch_deep1b && fetch deep1b &&
  step soar && timeout -k 10 900 python bench.py --config soar100m > $O/bench_soar100m_shard.json 2> $O/bench_soar100m_shard.err &&
  step deep1b && timeout -k 10 1000 python bench.py --config deep1b > $O/bench_deep1b_shard.json 2> $O/bench_deep1b_shard.err && step done ;;
d)
  step alone_deep1b && alone deep1b &&
  step stamps && timeout -k 10 300 python tools/phase_stamps.py 4 > $O/phases_glove.log 2>&1 &&
  step pmc_scan && KREGEX=lut16_scan_kernel timeout -k 10 600 bash tools/pmc_kernel.sh $O/pmc_scan_glove &&
  python tools/pmc_summary.py $O/pmc_scan_glove > $O/pmc_scan_glove.txt &&
  step pmc_seed && KREGEX=seed_tau_kernel timeout -k 10 600 bash tools/pmc_kernel.sh $O/pmc_seed_glove &&
  python tools/pmc_summary.py $O/pmc_seed_glove > $O/pmc_seed_glove.txt && step done ;;
esac
