#!/bin/bash
# Round-4 session P: cooperative 128-B line gathers with 8 / 4 / 2 lines (pages) per wave instruction, on
# tables inside and past the translation reach (3, 24, 96 GB).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
: > $OUT/gather_pages_r4p.jsonl
for gb in 3 24 96; do
  PROBE_PAGES=1 timeout -k 10 120 k-step_fm-index_amd/bin/gather_probe $gb 512 >> $OUT/gather_pages_r4p.jsonl 2>> $OUT/gather_pages_r4p.log || { tail -5 $OUT/gather_pages_r4p.log; exit 31; }
done
cat $OUT/gather_pages_r4p.jsonl
echo done
