set -o pipefail
mkdir -p gpurun_out
LIBS="scann_amd/lib/libscann_mi355x.so scann_amd/lib/exp/libseed_p16_u8.so scann_amd/lib/exp/libseed_p24_u8.so scann_amd/lib/exp/libseed_p16_u4.so" TAG=r03h.seed STEPS=200 bash tools/ab_libs.sh &&
timeout -k 10 900 python bench.py --config deep1b --steps 10 --warmup 2 --no-cpu-baseline --sweep-steps 8 > gpurun_out/r03h.deep.json 2> gpurun_out/r03h.deep.err
