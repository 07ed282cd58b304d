#!/bin/bash
# Round-1 session D: L2-locality experiments on task-mid: non-temporal deep
# steps (KFMI_NT_FROM) and suffix-ordered reads.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 python3 $R/scripts/sweep.py --backends task-mid --env "KFMI_NT_FROM=1000,2,4,5,6,8" --steps 5 > $OUT/sweep_nt.jsonl 2> $OUT/sweep_nt.log || exit 41
echo nt_done
timeout -k 10 400 python3 $R/scripts/sweep.py --backends task-mid,coop-mid --env "KFMI_NT_FROM=1000,5" --sort-suffix 16 --steps 5 > $OUT/sweep_sort.jsonl 2> $OUT/sweep_sort.log || exit 42
echo sort_done
