#!/bin/bash
# Round-2 session J: stream tests, then the mode x ISA sweep with the persistent cost model.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
cd /tmp
timeout -k 10 400 python3 -u $R/scripts/e2e_modes.py > $OUT/e2e_modes_r2k.jsonl 2> $OUT/e2e_modes_r2k.log || { tail -30 $OUT/e2e_modes_r2k.log; exit 33; }
cat $OUT/e2e_modes_r2k.jsonl
