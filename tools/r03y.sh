set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_many_leaves.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -q --timeout 250 --timeout-method thread > gpurun_out/r03y.tests.log 2>&1 &&
timeout -k 10 240 python tools/phase_stamps.py > gpurun_out/r03y.phase.log 2>&1 &&
LIBS="scann_amd/lib/libscann_mi355x_head.so scann_amd/lib/libscann_mi355x.so" TAG=ab_y STEPS=300 bash tools/ab_libs.sh
