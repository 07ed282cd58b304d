#!/bin/bash
# Round-2 session A: upside of batch order -- task-mid / coop-mid LF time with the
# 10M reads ordered by their last 0/16/24/32 bases (host-side order; the device
# reorder is only worth building if this shows a clear gain).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 500 python3 -u $R/scripts/sweep.py --backends task-mid,coop-mid --sort-suffix 0,16,24,32 --steps 10 > $OUT/sweep_sort_r2a.jsonl 2> $OUT/sweep_sort_r2a.log || { tail -30 $OUT/sweep_sort_r2a.log; exit 32; }
cat $OUT/sweep_sort_r2a.jsonl
