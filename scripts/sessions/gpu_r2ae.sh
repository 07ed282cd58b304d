#!/bin/bash
# Round-2 session AE: per-thread search streams -- concurrency tests, then
# small batches from 1-8 host threads.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_concurrent_search.py tests/test_stream.py tests/test_groups.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r2ae.log 2>&1 || { tail -40 $OUT/gpu_tests_r2ae.log; exit 31; }
tail -2 $OUT/gpu_tests_r2ae.log
cd /tmp
timeout -k 10 700 python3 -u $R/scripts/batch_sweep.py > $OUT/batch_r2ae.jsonl 2> $OUT/batch_r2ae.log || { tail -30 $OUT/batch_r2ae.log; exit 32; }
grep threads $OUT/batch_r2ae.jsonl
