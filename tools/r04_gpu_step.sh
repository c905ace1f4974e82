# one-off steps of this round (run through gpurun from the repo root)
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04zp}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T.tests.log 2>&1 || exit $?
LIBS="scann_amd/lib/libscann_mi355x_r03.so scann_amd/lib/libscann_mi355x_prev.so scann_amd/lib/libscann_mi355x.so" TAG=${T}_glove STEPS=200 bash tools/ab_libs.sh &&
LIBS="scann_amd/lib/libscann_mi355x_prev.so scann_amd/lib/libscann_mi355x.so" TAG=${T}_sift STEPS=200 BENCH_ARGS="--config sift" bash tools/ab_libs.sh &&
LIBS="scann_amd/lib/libscann_mi355x_prev.so scann_amd/lib/libscann_mi355x.so" TAG=${T}_deep STEPS=20 LIMIT=400 BENCH_ARGS="--config deep1b --no-parity --warmup 3" bash tools/ab_libs.sh
