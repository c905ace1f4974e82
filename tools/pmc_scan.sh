#!/bin/bash
# PMC passes over the scan kernel (one rocprofv3 run per counter group; no
# trace domains combined with --pmc).  Run on the GPU box from the repo root:
#   bash tools/pmc_scan.sh <tune.py config, e.g. 4096,2,0,32> <outdir> ["grp1;grp2;..."]
set -e
CFG=${1:-4096,2,0,32}
OUT=${2:-gpurun_out/pmc_scan}
PMCG=${3:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE;SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU;SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS;SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_WAVES SQ_BUSY_CYCLES"}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
IFS=';' read -ra GRP <<< "$PMCG"
for grp in "${GRP[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$ROOT/$OUT/p$i" -o run \
    --kernel-include-regex "lut16_scan" -- python3 "$ROOT/tools/tune.py" "$CFG" > "$ROOT/$OUT/p$i.log" 2>&1
done
