set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --config sift --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/r03x.sift.json 2> gpurun_out/r03x.sift.err && \
timeout -k 10 600 python bench.py --config soar100m --steps 30 --warmup 5 --cpu-threads 16 > gpurun_out/r03x.soar.json 2> gpurun_out/r03x.soar.err && \
CFG=deep1b bash tools/prof_config.sh gpurun_out/r03x.profd
