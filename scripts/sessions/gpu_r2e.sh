#!/bin/bash
# Round-2 session E: the in-call reorder (KFMI_REORDER) -- parity, then the
# 3 Gbase A/B with per-kernel times under rocprofv3.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k reorder --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r2e.log 2>&1 || { tail -40 $OUT/gpu_tests_r2e.log; exit 31; }
tail -2 $OUT/gpu_tests_r2e.log
cd /tmp
timeout -k 10 400 python3 -u $R/scripts/sweep.py --backends task-mid,task-ac,task-packed --env "KFMI_REORDER=0,1,0,1" --steps 10 > $OUT/sweep_reorder_r2e.jsonl 2> $OUT/sweep_reorder_r2e.log || { tail -30 $OUT/sweep_reorder_r2e.log; exit 32; }
cat $OUT/sweep_reorder_r2e.jsonl
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_r2e -o sw --output-format csv -- python3 $R/scripts/sweep.py --backends task-mid --env "KFMI_REORDER=0,1" --steps 10 > $OUT/prof_sweep_r2e.jsonl 2> $OUT/prof_sweep_r2e.log || { tail -30 $OUT/prof_sweep_r2e.log; exit 33; }
cat $(find $OUT/prof_r2e -name "*kernel_stats.csv") | cut -c1-250 | head -20
