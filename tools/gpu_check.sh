#!/bin/bash
# One GPU-box pass over the round's evidence (run through gpurun from the
# repo root): the -m gpu suite on the product library, smoke(), the bench
# line, and -- with DIAG=1 -- the same suite once more on the diagnostic
# library (device index checks on every computed index) plus the phase-stamp
# tool.  Every GPU step has its own time limit and the steps are chained
# with && (nothing runs after a failure).  Output: gpurun_out/$TAG.*
set -o pipefail
TAG=${TAG:-check}
O=gpurun_out
mkdir -p $O
PYTEST="python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread"
step() { echo "[gpu_check] $(date +%T) $*" >&2; }
run_diag() {
  step "diag suite"
  SMX_LIB=scann_amd/lib/libscann_mi355x_diag.so timeout -k 10 600 $PYTEST \
      > $O/$TAG.diag_tests.log 2>&1 &&
  step "phase stamps" &&
  timeout -k 10 240 python tools/phase_stamps.py > $O/$TAG.phase.log 2>&1
}
if [ -n "${MB:-}" ]; then
  step "microbench $MB"
  timeout -k 10 120 $MB > $O/$TAG.mb.log 2>&1 || { step "microbench failed"; exit 1; }
fi
step "product suite" &&
timeout -k 10 600 $PYTEST > $O/$TAG.tests.log 2>&1 &&
step "smoke" &&
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/$TAG.smoke.log 2>&1 &&
step "bench" &&
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $O/$TAG.bench.json 2> $O/$TAG.bench.err &&
if [ "${DIAG:-0}" = "1" ]; then run_diag; fi
rc=$?
step "done rc=$rc"
exit $rc
