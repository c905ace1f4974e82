#!/bin/bash
# Round-5 shard lines: configs[3] (soar100m) and configs[4] (deep1b), rank 0
# of the 8-way split on one GPU, three batches in flight, parity on the shard
# engine vs the oracle, CPU baseline.
set -o pipefail
O=gpurun_out/${TAG:-r05h}
mkdir -p $O
step() { echo "[r05_h] $(date +%T) $*" >&2; }
step soar && timeout -k 10 900 python bench.py --config soar100m > $O/bench_soar100m_shard.json 2> $O/bench_soar100m_shard.err &&
step deep1b && timeout -k 10 1000 python bench.py --config deep1b > $O/bench_deep1b_shard.json 2> $O/bench_deep1b_shard.err &&
step done
