#!/bin/bash
# Round-2 session AL (AK re-run with 6 slots and the greedy mode 4 beside): streamed search with the batch-balanced transfer mix
# (adaptive mode packs the share f of reads that equalises host and link time).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_stream.py tests/test_concurrent_search.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r2al.log 2>&1 || { tail -40 $OUT/gpu_tests_r2al.log; exit 31; }
tail -1 $OUT/gpu_tests_r2al.log
cd /tmp
E2E_SLOTS=3,6 E2E_MODES=1,2,4,0 timeout -k 10 800 python3 -u $R/scripts/e2e_modes.py > $OUT/e2e_modes_r2al.jsonl 2> $OUT/e2e_modes_r2al.log || { tail -30 $OUT/e2e_modes_r2al.log; exit 32; }
cut -c1-220 $OUT/e2e_modes_r2al.jsonl
