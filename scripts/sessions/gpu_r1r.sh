#!/bin/bash
# Round-1 session R: ftab 16 bases (34 GB table) after the grid-stride fix; locate tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests/test_locate.py tests/test_gpu_parity.py -m gpu -x -q -k "locate or ftab" --timeout 300 --timeout-method thread > $OUT/gpu_tests_r.log 2>&1 || { echo tests_failed; tail -40 $OUT/gpu_tests_r.log; exit 21; }
tail -1 $OUT/gpu_tests_r.log
cd /tmp
timeout -k 10 500 python3 $R/scripts/sweep.py --backends task-mid --env "KFMI_FTAB=14,16" --steps 10 > $OUT/sweep_ftab16.jsonl 2> $OUT/sweep_ftab16.log || exit 31
cat $OUT/sweep_ftab16.jsonl
