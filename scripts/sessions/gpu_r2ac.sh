#!/bin/bash
# Round-2 session AC: cooperative (LDS-staged) locate walk on MID lines --
# locate tests, then rate 1/8/32 with and without it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_locate.py tests/test_kstep3.py tests/test_kstep4.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r2ac.log 2>&1 || { tail -40 $OUT/gpu_tests_r2ac.log; exit 31; }
tail -2 $OUT/gpu_tests_r2ac.log
cd /tmp
timeout -k 10 600 python3 -u $R/scripts/locate_sweep.py --rates 1,8,32 --backends task-mid --coop 0,1,0,1 > $OUT/locate_r2ac.jsonl 2> $OUT/locate_r2ac.log || { tail -30 $OUT/locate_r2ac.log; exit 32; }
cat $OUT/locate_r2ac.jsonl
