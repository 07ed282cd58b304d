#!/bin/bash
# Round-2 session Q: K=4 grouped-counter backends -- tests, then 3 Gbase timings.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_kstep4.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r2q.log 2>&1 || { tail -40 $OUT/gpu_tests_r2q.log; exit 31; }
tail -2 $OUT/gpu_tests_r2q.log
cd /tmp
free -g | head -2
timeout -k 10 600 python3 -u $R/scripts/sweep.py --k 4 --backends coop-grp,task-grp --steps 10 > $OUT/sweep_grp_r2q.jsonl 2> $OUT/sweep_grp_r2q.log || { tail -30 $OUT/sweep_grp_r2q.log; exit 32; }
cat $OUT/sweep_grp_r2q.jsonl
