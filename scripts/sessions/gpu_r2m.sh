#!/bin/bash
# Round-2 session M: ingest tests (host + device parse), then the full GPU suite and the default bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_ingest.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r2m_ingest.log 2>&1 || { tail -40 $OUT/gpu_tests_r2m_ingest.log; exit 31; }
tail -2 $OUT/gpu_tests_r2m_ingest.log
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r2m.log 2>&1 || { tail -40 $OUT/gpu_tests_r2m.log; exit 32; }
tail -2 $OUT/gpu_tests_r2m.log
cd /tmp
timeout -k 10 400 python3 $R/bench.py > $OUT/bench_r2m.json 2> $OUT/bench_r2m.log || { tail -30 $OUT/bench_r2m.log; exit 33; }
cut -c1-300 $OUT/bench_r2m.json
