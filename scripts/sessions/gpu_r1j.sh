#!/bin/bash
# Round-1 session J: one-round-trip locate walk -- locate tests, rate sweep.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests/test_locate.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_locate_j.log 2>&1 || { echo locate_tests_failed; tail -40 $OUT/gpu_tests_locate_j.log; exit 21; }
tail -1 $OUT/gpu_tests_locate_j.log
cd /tmp
timeout -k 10 600 python3 $R/scripts/locate_sweep.py --rates 1,8,32 --regs 0 > $OUT/locate_sweep.jsonl 2> $OUT/locate_sweep.log || { tail -20 $OUT/locate_sweep.log; exit 31; }
cat $OUT/locate_sweep.jsonl
