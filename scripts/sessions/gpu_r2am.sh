#!/bin/bash
# Round-2 session AM: 6 stream slots with the per-chunk rule; slot sweep
# (4/6/8, default mode), stream tests, then the default bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_stream.py tests/test_concurrent_search.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r2am.log 2>&1 || { tail -40 $OUT/gpu_tests_r2am.log; exit 31; }
tail -1 $OUT/gpu_tests_r2am.log
cd /tmp
E2E_SLOTS=4,6,8 E2E_MODES=2,1 timeout -k 10 600 python3 -u $R/scripts/e2e_modes.py > $OUT/e2e_modes_r2am.jsonl 2> $OUT/e2e_modes_r2am.log || { tail -30 $OUT/e2e_modes_r2am.log; exit 32; }
cut -c1-140 $OUT/e2e_modes_r2am.jsonl
timeout -k 10 600 python3 $R/bench.py > $OUT/bench_r2am.json 2> $OUT/bench_r2am.log || { tail -30 $OUT/bench_r2am.log; exit 33; }
cut -c1-300 $OUT/bench_r2am.json
