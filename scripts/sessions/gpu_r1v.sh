#!/bin/bash
# Round-1 session V: ftab on the coop kernels -- parity + sweep.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k ftab --timeout 300 --timeout-method thread > $OUT/gpu_tests_v.log 2>&1 || { echo tests_failed; tail -40 $OUT/gpu_tests_v.log; exit 21; }
tail -1 $OUT/gpu_tests_v.log
cd /tmp
timeout -k 10 500 python3 $R/scripts/sweep.py --backends coop-mid,coop-ac128,task-ac --env "KFMI_FTAB=0,14" --steps 10 > $OUT/sweep_ftab_coop.jsonl 2> $OUT/sweep_ftab_coop.log || exit 31
cat $OUT/sweep_ftab_coop.jsonl | cut -c1-140
