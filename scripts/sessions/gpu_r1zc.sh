#!/bin/bash
# Round-1 session ZC: host-packed streaming, host thread count sweep (with host / wait time split).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp
for t in 1 4 8 16; do
  echo "threads $t"
  KFMI_HOST_THREADS=$t timeout -k 10 200 python3 $R/scripts/e2e_sweep.py --chunks 262144,524288,1048576 > $OUT/e2e_sweep_t$t.jsonl 2> $OUT/e2e_sweep_t$t.log || exit 31
  cat $OUT/e2e_sweep_t$t.jsonl
done
