# one-off steps of this round (run through gpurun from the repo root)
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04y}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T.tests.log 2>&1 || exit $?
timeout -k 10 240 python tools/phase_stamps.py > gpurun_out/$T.phase.log 2>&1 &&
LIBS="scann_amd/lib/libscann_mi355x_r03.so scann_amd/lib/libscann_mi355x.so" TAG=${T}_ab STEPS=200 bash tools/ab_libs.sh
