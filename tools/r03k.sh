set -o pipefail
mkdir -p gpurun_out
TAG=r03k bash tools/gpu_check.sh && \
timeout -k 10 900 bash tools/profile_bench.sh gpurun_out/r03k.prof && \
timeout -k 10 600 python bench.py --config deep1b --steps 10 --warmup 2 --no-cpu-baseline --sweep-steps 8 > gpurun_out/r03k.deep.json 2> gpurun_out/r03k.deep.err
