#!/bin/bash
# Round-2 session AJ: split-issue gathers at 150 bp (16-word fused kernel):
# forced 1 / 4 and the default rule ("" = unset), K=2 and K=4.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 python3 -u $R/scripts/sweep.py --qlen 150 --backends task-mid,task,task-ac128,task-ac --env "KFMI_SPLIT=1,4," --steps 10 > $OUT/sweep_split150_r2aj.jsonl 2> $OUT/sweep_split150_r2aj.log || { tail -30 $OUT/sweep_split150_r2aj.log; exit 31; }
timeout -k 10 400 python3 -u $R/scripts/sweep.py --k 4 --qlen 150 --backends task-grp --env "KFMI_SPLIT=1,4" --steps 10 >> $OUT/sweep_split150_r2aj.jsonl 2>> $OUT/sweep_split150_r2aj.log || { tail -30 $OUT/sweep_split150_r2aj.log; exit 32; }
cut -c1-150 $OUT/sweep_split150_r2aj.jsonl
