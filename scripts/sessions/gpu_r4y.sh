#!/bin/bash
# Round-4 session Y: searchIndexCPU with the host index image on 2 MB vs 4 KB pages (3 Gbase, 16 threads),
# alternating processes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
: > $OUT/cpu_hugepage_r4y.jsonl
for hp in 1 0 1 0; do
  KFMI_HUGEPAGES=$hp timeout -k 10 300 python3 scripts/cpu_hugepage_probe.py >> $OUT/cpu_hugepage_r4y.jsonl 2>> $OUT/cpu_hugepage_r4y.log || { tail -20 $OUT/cpu_hugepage_r4y.log; exit 31; }
done
cat $OUT/cpu_hugepage_r4y.jsonl
echo done
