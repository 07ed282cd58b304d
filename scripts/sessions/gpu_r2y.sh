#!/bin/bash
# Round-2 session Y: drop-in driver on a reference-built K=4 index; kernel
# trace + stats of the K=4 sweep (coop-grp, with and without ftab16).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_dropin.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r2y.log 2>&1 || { tail -40 $OUT/gpu_tests_r2y.log; exit 31; }
tail -2 $OUT/gpu_tests_r2y.log
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_grp_r2y -o p --output-format csv -- python3 $R/scripts/sweep.py --k 4 --backends coop-grp --env "KFMI_FTAB=0,16" --steps 10 > $OUT/prof_grp_r2y.jsonl 2> $OUT/prof_grp_r2y.log || { tail -30 $OUT/prof_grp_r2y.log; exit 32; }
cat $OUT/prof_grp_r2y.jsonl
head -6 $OUT/prof_grp_r2y/p_kernel_stats.csv | cut -c1-250
