set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_many_leaves.py tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -v --timeout 250 --timeout-method thread > gpurun_out/r03r.tests.log 2>&1 &&
CFG=deep1b bash tools/prof_config.sh gpurun_out/profr
