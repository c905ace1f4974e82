set -o pipefail
mkdir -p gpurun_out
SMX_LIB=scann_amd/lib/exp/libsdwa2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r03o.parity.log 2>&1 &&
LIBS="scann_amd/lib/exp/libsdwa.so scann_amd/lib/exp/libsdwa2.so" TAG=r03o STEPS=300 bash tools/ab_libs.sh
