#!/bin/bash
# Front-end timing probes on the diagnostic library (tools/tune.py lines):
# fused vs separate front end, the work-list / scatter parts of the fused
# launch (SMX_WLS_PART), and the seed-leaf count.
set -o pipefail
O=gpurun_out/${TAG:-probe}
mkdir -p $O
step() { echo "[probe] $(date +%T) $*" >&2; }
step "fused, seed sweep" &&
SMX_FUSED_FRONT=1 timeout -k 10 300 python3 tools/tune.py 0,4,0,20 0,1,0,20 0,2,0,20 0,3,0,20 0,4,0,32 0,4,0,64 > $O/fused.log 2>&1 &&
step "separate" &&
SMX_FUSED_FRONT=0 timeout -k 10 200 python3 tools/tune.py 0,4,0,20 0,2,0,20 > $O/separate.log 2>&1 &&
step "part 1" &&
SMX_FUSED_FRONT=1 SMX_WLS_PART=1 timeout -k 10 200 python3 tools/tune.py 0,4,0,20 > $O/part1.log 2>&1 &&
step "part 2" &&
SMX_FUSED_FRONT=1 SMX_WLS_PART=2 timeout -k 10 200 python3 tools/tune.py 0,4,0,20 > $O/part2.log 2>&1
rc=$?
step "done rc=$rc"
exit $rc
