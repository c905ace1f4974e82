# one-off steps of this round (run through gpurun from the repo root)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r04k.tests.log 2>&1
rc=$?
echo "tests rc=$rc" >&2
[ $rc -le 1 ] || exit $rc
LIBS="scann_amd/lib/libscann_mi355x_r03.so scann_amd/lib/libscann_mi355x.so" TAG=r04k_ab STEPS=200 bash tools/ab_libs.sh
