# one-off steps of this round (run through gpurun from the repo root)
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04r}
timeout -k 10 400 python -u -m pytest tests/test_gpu_paths.py -x -v --timeout 200 --timeout-method thread > gpurun_out/$T.tests.log 2>&1 || exit $?
ENVS="SMX_SEED_MFMA=0 SMX_SEED_MFMA=1" TAG=${T}_trace bash tools/trace_env.sh
