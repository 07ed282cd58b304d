#!/bin/bash
# Round-3 session N: fetch forms 1, 4 (C++ split), 6-8 (asm, empty parts skipped: 4, 2, 1 groups)
# four groups with a wait per group (5), asm four groups one wait (6), asm one
# group (1) -- at 100 bp and 150 bp (config #5's read length).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 700 python3 -u $R/scripts/sweep.py --backends task,task-ac,task-mid --env "KFMI_SPLIT=1,4,6,7,8" --steps 10 > $OUT/sweep_r3n.jsonl 2> $OUT/sweep_r3n.log || { tail -30 $OUT/sweep_r3n.log; exit 33; }
cut -c1-170 $OUT/sweep_r3n.jsonl
timeout -k 10 700 python3 -u $R/scripts/sweep.py --qlen 150 --backends task-mid,task-ac --env "KFMI_SPLIT=1,4,7,8" --steps 10 > $OUT/sweep150_r3n.jsonl 2> $OUT/sweep150_r3n.log || { tail -30 $OUT/sweep150_r3n.log; exit 34; }
cut -c1-170 $OUT/sweep150_r3n.jsonl
