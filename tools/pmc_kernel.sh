#!/bin/bash
# PMC passes (no trace) over one kernel of the bench workload (GPU box, repo root):
#   KREGEX=seed_tau_kernel [BENCH_ARGS="--config sift"] bash tools/pmc_kernel.sh <outdir>
# then: python tools/pmc_summary.py <outdir>
set -e
OUT=${1:-gpurun_out/pmck}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_WAVES SQ_INSTS_SALU" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d "$ROOT/$OUT/p$i" -o run \
    --kernel-include-regex "${KREGEX:-seed_tau_kernel}" -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-sweep --no-parity --no-latency --no-stages --steps 20 ${BENCH_ARGS:-} \
    > "$ROOT/$OUT/p$i.log" 2>&1
done
