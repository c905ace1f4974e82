set -o pipefail
mkdir -p gpurun_out
TAG=r03p bash tools/gpu_check.sh && \
timeout -k 10 900 bash tools/profile_bench.sh gpurun_out/r03p.prof && \
timeout -k 10 400 python bench.py --config sift --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/r03p.sift.json 2> gpurun_out/r03p.sift.err && \
timeout -k 10 600 python bench.py --config soar100m --steps 30 --warmup 5 --cpu-threads 16 > gpurun_out/r03p.soar.json 2> gpurun_out/r03p.soar.err
