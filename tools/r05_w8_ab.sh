#!/bin/bash
# Scan waves per workgroup (SMX_SCAN_WAVES build) against the product
# library, interleaved, glove; the 8-wave build also at 4 batches in flight.
set -o pipefail
O=gpurun_out/${TAG:-r05w8b}
mkdir -p $O
step() { echo "[r05_w8_ab] $(date +%T) $*" >&2; }
A="--steps 300 --warmup 20 --no-cpu-baseline --no-sweep --no-parity"
for rep in 1 2 3; do
  step "w12 rep $rep" && SMX_LIB=scann_amd/lib/libscann_mi355x.so timeout -k 10 300 python3 bench.py $A >> $O/w12.json 2>> $O/bench.err &&
  step "w8 rep $rep" && SMX_LIB=scann_amd/lib/libscann_mi355x_w8.so timeout -k 10 300 python3 bench.py $A >> $O/w8.json 2>> $O/bench.err &&
  step "w8 fl4 rep $rep" && SMX_LIB=scann_amd/lib/libscann_mi355x_w8.so timeout -k 10 300 python3 bench.py $A --in-flight 4 >> $O/w8_fl4.json 2>> $O/bench.err &&
  step "w12 sift rep $rep" && SMX_LIB=scann_amd/lib/libscann_mi355x.so timeout -k 10 300 python3 bench.py $A --config sift >> $O/w12_sift.json 2>> $O/bench.err &&
  step "w8 sift rep $rep" && SMX_LIB=scann_amd/lib/libscann_mi355x_w8.so timeout -k 10 300 python3 bench.py $A --config sift >> $O/w8_sift.json 2>> $O/bench.err || exit 1
done
step done
