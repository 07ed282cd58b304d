#!/bin/bash
# Round-1 session G: LDS-staged fused packing -- GPU tests, A/B sweep, bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_g.log 2>&1 || { echo tests_failed; tail -30 $OUT/gpu_tests_g.log; exit 21; }
tail -1 $OUT/gpu_tests_g.log
cd /tmp
timeout -k 10 400 python3 $R/scripts/sweep.py --backends task-mid,task-ac --env "KFMI_FUSED=0,1" --steps 5 > $OUT/sweep_fused_g.jsonl 2> $OUT/sweep_fused_g.log || exit 31
timeout -k 10 400 python3 $R/scripts/sweep.py --backends task-mid --env "KFMI_FUSED=0,1" --qlen 150 --steps 5 > $OUT/sweep_fused_g150.jsonl 2> $OUT/sweep_fused_g150.log || exit 32
cat $OUT/sweep_fused_g.jsonl $OUT/sweep_fused_g150.jsonl
