#!/bin/bash
# Round profile of the bench workload (run on the GPU box from the repo root):
#   [BENCH_ARGS="--config sift"] bash tools/profile_bench.sh <outdir>
# 1) rocprofv3 kernel trace + stats of bench.py (no PMC in this pass; the
#    timed region only: --no-latency --no-stages skip the one-at-a-time
#    timing and the per-stage replay, so the trace's scan launches are the
#    timed region's, whose HIP-event average the bench line reports);
# 2) one PMC pass per counter group over the scan kernel: FETCH_SIZE (HBM
#    traffic, gfx950 x2 correction in tools/pmc_traffic.py), WRITE_SIZE, the
#    SQ busy/wait counters and the LDS counters.
set -e
OUT=${1:-gpurun_out/prof}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/trace" -o run \
  -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-sweep --no-parity --no-latency --no-stages --steps 200 ${BENCH_ARGS:-} > "$ROOT/$OUT/bench_traced.json" 2> "$ROOT/$OUT/bench_traced.err"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_WAVES SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d "$ROOT/$OUT/pmc$i" -o run \
    --kernel-include-regex "lut16_scan_kernel" -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-sweep --no-parity --steps 20 ${BENCH_ARGS:-} \
    > "$ROOT/$OUT/pmc$i.log" 2>&1
done
