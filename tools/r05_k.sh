#!/bin/bash
# Cross-tile operand prefetch: parity suites on the new scan, then a same-box
# A/B against the previous library (glove; isolated scan in stage_ms).
set -o pipefail
O=gpurun_out/${TAG:-r05k}
mkdir -p $O
step() { echo "[r05_k] $(date +%T) $*" >&2; }
step tests && timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_paths.py tests/test_gpu_configs.py tests/test_gpu_streams.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 &&
step libs && TAG=$(basename $O)/libs LIBS="scann_amd/lib/libscann_mi355x_base.so scann_amd/lib/libscann_mi355x.so" STEPS=300 bash tools/ab_libs.sh &&
step done
