set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/topl_stamps.py 400 > gpurun_out/topl_stamps.log 2>&1 &&
timeout -k 10 200 python tools/topl_stamps.py 2000 >> gpurun_out/topl_stamps.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/r03t.tests.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03t.glove.json 2> gpurun_out/r03t.glove.err &&
timeout -k 10 700 python bench.py --config deep1b --steps 10 --warmup 2 --no-cpu-baseline --sweep-steps 8 > gpurun_out/r03t.deep.json 2> gpurun_out/r03t.deep.err
