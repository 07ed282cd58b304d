#!/bin/bash
# Round-1 session E: the K=1 variants (Task-1Step / Coop-1Step),
# the d sweep {192,448,960} and 150-bp reads (config #5 shape)
# on the 3 Gbase index.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
export TMPDIR=/tmp
cd /tmp
ALL=task,coop,task-ac,coop-ac,task-packed,coop-packed,task-mid,coop-mid
timeout -k 10 400 python3 $R/scripts/sweep.py --k 1 --d 64 --backends $ALL --steps 5 > $OUT/sweep_k1.jsonl 2> $OUT/sweep_k1.log || exit 41
echo k1_done
for D in 192 448 960; do
  timeout -k 10 400 python3 $R/scripts/sweep.py --k 2 --d $D --backends $ALL --steps 5 > $OUT/sweep_d$D.jsonl 2> $OUT/sweep_d$D.log || exit 42
  echo d${D}_done
done
timeout -k 10 400 python3 $R/scripts/sweep.py --k 2 --d 64 --qlen 150 --backends task-mid,coop-mid,task-ac --steps 5 > $OUT/sweep_q150.jsonl 2> $OUT/sweep_q150.log || exit 43
echo q150_done
