#!/bin/bash
# Round-2 session BF: K = 4 results located through a K = 2 companion index
# (test_kstep4.py), plus the K = 3 tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 500 python3 -u -m pytest tests/test_kstep4.py tests/test_kstep3.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r2bf.log 2>&1 || { tail -40 $OUT/gpu_tests_r2bf.log; exit 31; }
tail -2 $OUT/gpu_tests_r2bf.log
