#!/bin/bash
# Round-1 session F: full GPU test suite + smoke on the fused-pack build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo tests_failed; tail -30 $OUT/gpu_tests.log; exit 21; }
tail -3 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke_failed; tail -20 $OUT/smoke.log; exit 22; }
tail -2 $OUT/smoke.log
