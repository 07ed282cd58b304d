#!/bin/bash
# Round-2 session AH: split-issue gathers (KFMI_SPLIT=4: per-lane loads as 4
# exec-masked groups of 16 lanes) on the task kernels, 3 Gbase, 10M x 100 bp.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 python3 -u $R/scripts/sweep.py --backends task-mid,task,task-ac128,task-ac,task-packed,task-ac-mid --env "KFMI_SPLIT=1,4" --steps 10 > $OUT/sweep_split_r2ah.jsonl 2> $OUT/sweep_split_r2ah.log || { tail -30 $OUT/sweep_split_r2ah.log; exit 31; }
timeout -k 10 300 python3 -u $R/scripts/sweep.py --backends task-mid --env "KFMI_FTAB=14,16;KFMI_SPLIT=1,4" --steps 10 > $OUT/sweep_split_ftab_r2ah.jsonl 2> $OUT/sweep_split_ftab_r2ah.log || { tail -30 $OUT/sweep_split_ftab_r2ah.log; exit 32; }
timeout -k 10 400 python3 -u $R/scripts/sweep.py --k 4 --backends task-grp,coop-grp --env "KFMI_SPLIT=1,4" --steps 10 > $OUT/sweep_split_grp_r2ah.jsonl 2> $OUT/sweep_split_grp_r2ah.log || { tail -30 $OUT/sweep_split_grp_r2ah.log; exit 33; }
cut -c1-200 $OUT/sweep_split*_r2ah.jsonl
