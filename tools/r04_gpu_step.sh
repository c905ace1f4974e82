# one-off steps of this round (run through gpurun from the repo root)
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04zn}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T.tests.log 2>&1 || exit $?
ENVS="SMX_LIB=scann_amd/lib/libscann_mi355x_r03.so SMX_LIB=scann_amd/lib/libscann_mi355x.so" TAG=${T}_trace bash tools/trace_env.sh &&
LIBS="scann_amd/lib/libscann_mi355x_r03.so scann_amd/lib/libscann_mi355x.so" TAG=${T}_glove STEPS=200 bash tools/ab_libs.sh
