#!/bin/bash
# Round-2 session G: streamed search -- tests (incl. mixed chunk modes) and the
# mode x ISA measurement on 3 Gbase.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_stream.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r2g.log 2>&1 || { tail -40 $OUT/gpu_tests_r2g.log; exit 31; }
tail -2 $OUT/gpu_tests_r2g.log
cd /tmp
timeout -k 10 400 python3 -u $R/scripts/e2e_modes.py > $OUT/e2e_modes_r2g.jsonl 2> $OUT/e2e_modes_r2g.log || { tail -30 $OUT/e2e_modes_r2g.log; exit 32; }
cat $OUT/e2e_modes_r2g.jsonl
