#!/bin/bash
# Round-2 session D: GPU builder tests (device prefix-doubling tie resolution).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_builder.py -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r2d.log 2>&1 || { tail -40 $OUT/gpu_tests_r2d.log; exit 31; }
grep -E "repeat-rich|passed|failed" $OUT/gpu_tests_r2d.log
