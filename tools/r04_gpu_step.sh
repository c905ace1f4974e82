# one-off steps of this round (run through gpurun from the repo root)
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04zb}
ENVS="SMX_SERIAL_WORKLIST=0 SMX_SERIAL_WORKLIST=1" TAG=${T}_soar STEPS=30 LIMIT=300 BENCH_ARGS="--config soar100m --no-parity --warmup 5" bash tools/ab_env.sh &&
ENVS="SMX_SERIAL_WORKLIST=0 SMX_SERIAL_WORKLIST=1" TAG=${T}_deep STEPS=20 LIMIT=400 BENCH_ARGS="--config deep1b --no-parity --warmup 3" bash tools/ab_env.sh
