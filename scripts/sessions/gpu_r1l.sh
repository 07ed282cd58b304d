#!/bin/bash
# Round-1 session L: AC128 layout (task-ac128/coop-ac128) -- full GPU tests + AC sweep.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_l.log 2>&1 || { echo tests_failed; tail -40 $OUT/gpu_tests_l.log; exit 21; }
tail -1 $OUT/gpu_tests_l.log
cd /tmp
timeout -k 10 500 python3 $R/scripts/sweep.py --backends task-ac,task-ac128,coop-ac,coop-ac128,task-mid --steps 10 > $OUT/sweep_ac128.jsonl 2> $OUT/sweep_ac128.log || exit 31
cat $OUT/sweep_ac128.jsonl
