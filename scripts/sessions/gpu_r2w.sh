#!/bin/bash
# Round-2 session W: K=4 + ftab jump start (coop-grp), and the implicit-default test.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_kstep4.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r2w.log 2>&1 || { tail -40 $OUT/gpu_tests_r2w.log; exit 31; }
tail -2 $OUT/gpu_tests_r2w.log
cd /tmp
timeout -k 10 600 python3 -u $R/scripts/sweep.py --k 4 --backends coop-grp --env "KFMI_FTAB=0,4,8,12,16" --steps 10 > $OUT/sweep_grp_ftab_r2w.jsonl 2> $OUT/sweep_grp_ftab_r2w.log || { tail -30 $OUT/sweep_grp_ftab_r2w.log; exit 32; }
cat $OUT/sweep_grp_ftab_r2w.jsonl
