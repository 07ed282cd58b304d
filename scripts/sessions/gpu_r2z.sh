#!/bin/bash
# Round-2 session Z: K=3 on the GPU -- tests, then 3 Gbase timings (coop-grp K=3
# at 99 / 100 / 150 bp).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_kstep3.py tests/test_kstep4.py tests/test_remainder.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r2z.log 2>&1 || { tail -40 $OUT/gpu_tests_r2z.log; exit 31; }
tail -2 $OUT/gpu_tests_r2z.log
cd /tmp
timeout -k 10 400 python3 -u $R/scripts/sweep.py --k 3 --backends coop-grp,task-grp --steps 10 > $OUT/sweep_k3_r2z.jsonl 2> $OUT/sweep_k3_r2z.log || { tail -30 $OUT/sweep_k3_r2z.log; exit 32; }
timeout -k 10 400 python3 -u $R/scripts/sweep.py --k 3 --qlen 150 --backends coop-grp --steps 10 >> $OUT/sweep_k3_r2z.jsonl 2>> $OUT/sweep_k3_r2z.log || { tail -30 $OUT/sweep_k3_r2z.log; exit 33; }
cat $OUT/sweep_k3_r2z.jsonl
