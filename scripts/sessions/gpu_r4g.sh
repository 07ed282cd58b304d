#!/bin/bash
# Round-4 session G: the streamed search's link estimate without the in-flight division -- stream
# GPU tests, then host contention at P = 1, 2, 4, 8 (7 rounds).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_stream.py -x -q --timeout 250 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r4g.log 2>&1 || { tail -40 $OUT/gpu_tests_r4g.log; exit 31; }
tail -2 $OUT/gpu_tests_r4g.log
cd /tmp
timeout -k 10 700 python3 -u $R/scripts/stream_contention.py --procs 1 2 4 8 --ref-size 300000000 --rounds 7 --out $OUT/stream_contention_r4g.jsonl > $OUT/stream_contention_r4g.log 2>&1 || { tail -30 $OUT/stream_contention_r4g.log; exit 32; }
tail -8 $OUT/stream_contention_r4g.log | cut -c1-200
echo done
