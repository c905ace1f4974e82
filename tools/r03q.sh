set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_many_leaves.py tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -v --timeout 250 --timeout-method thread > gpurun_out/r03q.tests.log 2>&1 &&
timeout -k 10 700 python bench.py --config deep1b --steps 10 --warmup 2 --no-cpu-baseline --sweep-steps 8 > gpurun_out/r03q.deep.json 2> gpurun_out/r03q.deep.err
