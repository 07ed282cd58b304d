#!/bin/bash
# Round-2 session AO: full-scale GPU tests incl. K = 4 on 3 Gbase (96 GB GRP, split and plain issue).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_fullscale.py -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider --durations=5 > $OUT/gpu_tests_r2ao.log 2>&1 || { tail -40 $OUT/gpu_tests_r2ao.log; exit 31; }
tail -12 $OUT/gpu_tests_r2ao.log
