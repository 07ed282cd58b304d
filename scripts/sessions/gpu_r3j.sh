#!/bin/bash
# Round-3 session J: split-issue 1 vs 4 for the reference-layout task kernels
# with line-local counting.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 python3 -u $R/scripts/sweep.py --backends task,task-ac,task-mid --env "KFMI_SPLIT=1,4" --steps 10 > $OUT/sweep_r3j.jsonl 2> $OUT/sweep_r3j.log || { tail -30 $OUT/sweep_r3j.log; exit 33; }
cut -c1-160 $OUT/sweep_r3j.jsonl
