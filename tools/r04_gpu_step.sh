# one-off steps of this round (run through gpurun from the repo root)
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04zd}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T.tests.log 2>&1 || exit $?
LIBS="scann_amd/lib/libscann_mi355x_prev.so scann_amd/lib/libscann_mi355x.so" TAG=${T}_glove STEPS=200 bash tools/ab_libs.sh &&
LIBS="scann_amd/lib/libscann_mi355x_prev.so scann_amd/lib/libscann_mi355x.so" TAG=${T}_soar STEPS=30 LIMIT=300 BENCH_ARGS="--config soar100m --no-parity --warmup 5" bash tools/ab_libs.sh
