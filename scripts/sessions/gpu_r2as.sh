#!/bin/bash
# Round-2 session AS: locate walk slots from a per-wave queue (chunks of a global
# counter) instead of the fixed i, i + stride order -- locate + group tests, then
# rate 8 / 32 on 3 Gbase, per-lane and cooperative walks (pos md5 vs r2ac).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_locate.py tests/test_groups.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r2as.log 2>&1 || { tail -40 $OUT/gpu_tests_r2as.log; exit 31; }
tail -2 $OUT/gpu_tests_r2as.log
cd /tmp
timeout -k 10 600 python3 -u $R/scripts/locate_sweep.py --rates 8,32 --backends task-mid,task-ac --coop 0,1,0,1 > $OUT/locate_r2as.jsonl 2> $OUT/locate_r2as.log || { tail -30 $OUT/locate_r2as.log; exit 32; }
cut -c1-220 $OUT/locate_r2as.jsonl
