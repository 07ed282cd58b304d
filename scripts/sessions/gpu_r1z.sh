#!/bin/bash
# Round-1 session Z: occupancy experiment on task-mid (extra LDS caps resident workgroups:
# 0 -> 8 waves/SIMD, 7000 -> 6 (20 KB/WG), 27000 -> 4 (40 KB), 67000 -> 2 (80 KB)).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp
timeout -k 10 500 python3 $R/scripts/sweep.py --backends task-mid --env "KFMI_LDS_PAD=0,7000,14000,27000,67000,0" --steps 10 > $OUT/sweep_occupancy.jsonl 2> $OUT/sweep_occupancy.log || exit 31
cat $OUT/sweep_occupancy.jsonl | cut -c1-130
