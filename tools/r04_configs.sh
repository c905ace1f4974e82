# Round-4 generated-config bench lines (gpurun, repo root): configs[3] and
# configs[4] (rank 0's shard, merge of 8 lists), with parity_vs_oracle,
# sweeps and the CPU baseline on the shard.
set -o pipefail
O=gpurun_out/${TAG:-r04g}
mkdir -p $O
step() { echo "[r04_configs] $(date +%T) $*" >&2; }
step soar && timeout -k 10 700 python bench.py --config soar100m --steps 30 --warmup 5 > $O/bench_soar100m_shard.json 2> $O/bench_soar100m_shard.err &&
step deep && timeout -k 10 900 python bench.py --config deep1b --steps 20 --warmup 3 > $O/bench_deep1b_shard.json 2> $O/bench_deep1b_shard.err &&
step done
