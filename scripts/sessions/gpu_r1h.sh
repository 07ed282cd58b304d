#!/bin/bash
# Round-1 session H: fused-packing A/B with longer runs, alternating order.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 500 python3 $R/scripts/sweep.py --backends task-mid --env "KFMI_FUSED=1,0,1,0" --steps 20 > $OUT/sweep_fused_h.jsonl 2> $OUT/sweep_fused_h.log || exit 31
cat $OUT/sweep_fused_h.jsonl
