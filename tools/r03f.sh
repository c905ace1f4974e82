set -o pipefail
mkdir -p gpurun_out
TAG=r03f bash tools/gpu_check.sh && \
timeout -k 10 900 bash tools/profile_bench.sh gpurun_out/r03f.prof
