#!/bin/bash
# Round-2 session AG: translation-reach probe -- per-lane gathers issued as G
# exec-masked instructions (64/G lanes each) on 3 / 6 / 24 GB tables.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp PROBE_MASK=1
for gb in 3 6 24; do
  echo "{\"table_GB\": $gb}" >> $OUT/gather_mask_r2ag.jsonl
  timeout -k 10 120 $R/k-step_fm-index_amd/bin/gather_probe $gb 256 >> $OUT/gather_mask_r2ag.jsonl || exit 31
done
cat $OUT/gather_mask_r2ag.jsonl
