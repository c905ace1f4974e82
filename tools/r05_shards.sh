#!/bin/bash
# Round-5 shard lines (gpurun, repo root): a FETCH_SIZE pass over the scan of
# configs[3] (soar100m) and configs[4] (deep1b) for their traffic records,
# then both lines (rank 0 of the 8-way split on one GPU, three batches in
# flight, parity on the shard engine vs the oracle, CPU baseline).
set -o pipefail
O=gpurun_out/${TAG:-r05x}
ROOT=$(pwd)
mkdir -p $O
step() { echo "[r05_shards] $(date +%T) $*" >&2; }
fetch() {   # <config>
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv \
    -d "$ROOT/$O/pmc_$1" -o run --kernel-include-regex "lut16_scan_kernel" -- python3 "$ROOT/bench.py" \
    --config $1 --no-cpu-baseline --no-sweep --no-parity --steps 20 > "$ROOT/$O/pmc_$1.log" 2>&1) &&
  python tools/pmc_traffic.py $O/pmc_$1/run_counter_collection.csv $1 > $O/traffic_$1.log &&
  cp profiles/scan_traffic_$1.json $O/
}
step fetch_soar && fetch soar100m &&
step fetch_deep1b && fetch deep1b &&
step soar && timeout -k 10 900 python bench.py --config soar100m > $O/bench_soar100m_shard.json 2> $O/bench_soar100m_shard.err &&
step deep1b && timeout -k 10 1000 python bench.py --config deep1b > $O/bench_deep1b_shard.json 2> $O/bench_deep1b_shard.err &&
step done
