set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_generate.py tests/test_gpu_generate.py tests/test_gpu_device_build.py -m gpu -v --timeout 250 --timeout-method thread > gpurun_out/r03g.tests.log 2>&1 &&
timeout -k 10 500 python bench.py --config soar100m --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r03g.soar.json 2> gpurun_out/r03g.soar.err &&
timeout -k 10 700 python bench.py --config deep1b --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r03g.deep.json 2> gpurun_out/r03g.deep.err
