#!/bin/bash
# Round-5 follow-up pass (gpurun, repo root): the GPU suite on the debug
# library (bounds checks, scan diagnostics, phase stamps), then the SIFT
# trace + PMC passes, its traffic record and the SIFT line carrying it.
set -o pipefail
O=gpurun_out/${TAG:-r05s}
mkdir -p $O
step() { echo "[r05_sift_diag] $(date +%T) $*" >&2; }
step diag && SMX_LIB=scann_amd/lib/libscann_mi355x_diag.so timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/diag_tests.log 2>&1 &&
step prof_sift && BENCH_ARGS="--config sift" timeout -k 10 900 bash tools/profile_bench.sh $O/prof_sift &&
step traffic && python tools/pmc_traffic.py $O/prof_sift/pmc1/run_counter_collection.csv sift > $O/traffic.log &&
cp profiles/scan_traffic_sift.json $O/scan_traffic_sift.json &&
step sift && timeout -k 10 600 python bench.py --config sift > $O/bench_sift.json 2> $O/bench_sift.err &&
step done
