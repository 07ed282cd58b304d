#!/bin/bash
# Round-3 session Y: the coop issue forms A/B without the order effect --
# 20 untimed searches per variant and two passes in alternating order
# (KFMI_COOP_ISSUE 1 0 0 1), K = 2 coop backends, then coop-grp at K = 4.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 python3 -u $R/scripts/sweep.py --backends coop-mid,coop-ac-mid,coop-ac128,coop,coop-ac --env "KFMI_COOP_ISSUE=1,0" --steps 10 --warmup 20 --repeat 2 > $OUT/sweep_r3y.jsonl 2> $OUT/sweep_r3y.log || { tail -30 $OUT/sweep_r3y.log; exit 33; }
cut -c1-150 $OUT/sweep_r3y.jsonl
timeout -k 10 600 python3 -u $R/scripts/sweep.py --k 4 --backends coop-grp,task-grp --env "KFMI_COOP_ISSUE=1,0" --steps 10 --warmup 20 --repeat 2 > $OUT/sweep_k4_r3y.jsonl 2> $OUT/sweep_k4_r3y.log || { tail -30 $OUT/sweep_k4_r3y.log; exit 34; }
cut -c1-150 $OUT/sweep_k4_r3y.jsonl
