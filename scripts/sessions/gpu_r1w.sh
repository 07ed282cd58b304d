#!/bin/bash
# Round-1 session W: fused packing in the coop kernels -- GPU suite + A/B sweep.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_w.log 2>&1 || { echo tests_failed; tail -40 $OUT/gpu_tests_w.log; exit 21; }
tail -1 $OUT/gpu_tests_w.log
cd /tmp
timeout -k 10 600 python3 $R/scripts/sweep.py --backends coop-mid,coop-ac128,task-mid --env "KFMI_FUSED=1,0,1" --steps 15 > $OUT/sweep_coop_fused.jsonl 2> $OUT/sweep_coop_fused.log || exit 31
timeout -k 10 400 python3 $R/scripts/sweep.py --backends coop-mid --env "KFMI_FUSED=1,0" --qlen 150 --steps 10 > $OUT/sweep_coop_fused_q150.jsonl 2> $OUT/sweep_coop_fused_q150.log || exit 32
cat $OUT/sweep_coop_fused.jsonl $OUT/sweep_coop_fused_q150.jsonl | cut -c1-150
