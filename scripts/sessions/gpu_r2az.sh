#!/bin/bash
# Round-2 session AZ: long reads up to the LDS limit (2558 bases searched, 2560
# rejected) and the stream / ingest tests after the bound fix.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_stream.py tests/test_ingest.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r2az.log 2>&1 || { tail -40 $OUT/gpu_tests_r2az.log; exit 31; }
tail -2 $OUT/gpu_tests_r2az.log
