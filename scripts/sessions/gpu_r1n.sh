#!/bin/bash
# Round-1 session N: translation reach vs allocation mode (gather_probe, 6 GB).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp
for M in default contig vmm; do
  echo "== alloc=$M 6GB" >> $OUT/probe_alloc.txt
  PROBE_ALLOC=$M timeout -k 10 120 $R/k-step_fm-index_amd/bin/gather_probe 6 256 >> $OUT/probe_alloc.txt 2>&1 || echo "mode $M failed rc=$?" >> $OUT/probe_alloc.txt
done
cat $OUT/probe_alloc.txt
