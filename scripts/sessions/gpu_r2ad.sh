#!/bin/bash
# Round-2 session AD: per-call cost vs batch size.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 python3 -u $R/scripts/batch_sweep.py > $OUT/batch_r2ad.jsonl 2> $OUT/batch_r2ad.log || { tail -30 $OUT/batch_r2ad.log; exit 32; }
cat $OUT/batch_r2ad.jsonl
