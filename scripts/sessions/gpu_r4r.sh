#!/bin/bash
# Round-4 session R: fused packing vs pack kernel + packed-input LF at 100 and 150 bp.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 400 python3 scripts/fused_sweep.py > $OUT/fused_sweep_r4r.jsonl 2> $OUT/fused_sweep_r4r.log || { tail -20 $OUT/fused_sweep_r4r.log; exit 31; }
cat $OUT/fused_sweep_r4r.jsonl
echo done
