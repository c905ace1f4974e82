# one-off steps of this round (run through gpurun from the repo root)
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04za}
timeout -k 10 600 python -u -m pytest tests/test_gpu_paths.py tests/test_gpu_workload_shards.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_shards.py -x -v --timeout 300 --timeout-method thread > gpurun_out/$T.tests.log 2>&1 || exit $?
ENVS="SMX_NARROW=3 SMX_NARROW=1" TAG=${T}_deep STEPS=20 LIMIT=400 BENCH_ARGS="--config deep1b --no-parity --warmup 3" bash tools/ab_env.sh &&
ENVS="SMX_NARROW=3 SMX_NARROW=1" TAG=${T}_soar STEPS=30 LIMIT=300 BENCH_ARGS="--config soar100m --no-parity --warmup 5" bash tools/ab_env.sh
