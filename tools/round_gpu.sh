#!/bin/bash
# One GPU-box pass of this round's measurements (run through gpurun from the
# repo root); every GPU step under its own time limit, chained with &&.
#   diag : the -m gpu suite on the diagnostic library (device index checks on
#          every computed index) + the phase-stamp tool, once;
#   prof : the round profile of the bench workload (tools/profile_bench.sh).
# STEPS="diag prof" selects; output under gpurun_out/$TAG.*
set -o pipefail
TAG=${TAG:-rg}
O=gpurun_out
mkdir -p $O
step() { echo "[round_gpu] $(date +%T) $*" >&2; }
PYTEST="python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread"
rc=0
for s in ${STEPS:-diag prof}; do
  case $s in
    diag)
      step "diag suite" &&
      SMX_LIB=scann_amd/lib/libscann_mi355x_diag.so timeout -k 10 600 $PYTEST \
          > $O/$TAG.diag_tests.log 2>&1 &&
      step "phase stamps" &&
      timeout -k 10 240 python tools/phase_stamps.py > $O/$TAG.phase.log 2>&1 || rc=1 ;;
    prof)
      step "profile" && timeout -k 10 900 bash tools/profile_bench.sh $O/$TAG.prof || rc=1 ;;
    tune)
      step "tune" && timeout -k 10 300 python tools/tune.py ${TUNE_ARGS:-4096,4,0,20 4096,4,32,20 4096,4,4,20 4096,4,2,20 4096,4,16,20 4096,4,0,20} \
          > $O/$TAG.tune.log 2>&1 || rc=1 ;;
    phase)
      step "phase stamps (timing lib)" && timeout -k 10 240 python tools/phase_stamps.py > $O/$TAG.phase.log 2>&1 || rc=1 ;;
    stamps)
      step "scan stamps (timing lib)" && timeout -k 10 240 python tools/scan_stamps.py 20 > $O/$TAG.stamps.log 2>&1 || rc=1 ;;
    bench)
      step "bench" && timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $O/$TAG.bench.json 2> $O/$TAG.bench.err || rc=1 ;;
  esac
  [ $rc -ne 0 ] && break
done
step "done rc=$rc"
exit $rc
