#!/bin/bash
# Round-2 session AR (re-entry check of the restored tree): full GPU suite, smoke(), default bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_r2ar.log 2>&1 || { tail -40 $OUT/gpu_tests_r2ar.log; exit 31; }
tail -2 $OUT/gpu_tests_r2ar.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_r2ar.log 2>&1 || { tail -30 $OUT/smoke_r2ar.log; exit 30; }
tail -2 $OUT/smoke_r2ar.log
cd /tmp
timeout -k 10 600 python3 $R/bench.py > $OUT/bench_r2ar.json 2> $OUT/bench_r2ar.log || { tail -30 $OUT/bench_r2ar.log; exit 32; }
cut -c1-400 $OUT/bench_r2ar.json
