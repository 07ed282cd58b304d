#!/bin/bash
# Round-1 session P: ftab jump start -- parity tests and sweep of the table size.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k ftab --timeout 300 --timeout-method thread > $OUT/gpu_tests_ftab.log 2>&1 || { echo ftab_tests_failed; tail -40 $OUT/gpu_tests_ftab.log; exit 21; }
tail -1 $OUT/gpu_tests_ftab.log
cd /tmp
timeout -k 10 500 python3 $R/scripts/sweep.py --backends task-mid,task-ac --env "KFMI_FTAB=0,8,10,12,14" --steps 10 > $OUT/sweep_ftab.jsonl 2> $OUT/sweep_ftab.log || exit 31
cat $OUT/sweep_ftab.jsonl
