#!/bin/bash
# Round-1 session M: random-line rate vs table size (TLB reach), gather_probe.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp
for GB in 1.5 3 4 4.5 6 8 12 24; do
  echo "== table_GB=$GB" >> $OUT/probe_tlb.txt
  timeout -k 10 120 $R/k-step_fm-index_amd/bin/gather_probe $GB 256 >> $OUT/probe_tlb.txt 2>&1 || exit 41
done
cat $OUT/probe_tlb.txt
