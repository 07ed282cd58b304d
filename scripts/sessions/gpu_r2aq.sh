#!/bin/bash
# Round-2 session AQ: split-issue gathers in the per-lane locate walk --
# parity tests, then rate-32 locate at split 1 / 4 (K = 2 layouts, K = 4 GRP).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_locate.py tests/test_kstep4.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r2aq.log 2>&1 || { tail -40 $OUT/gpu_tests_r2aq.log; exit 31; }
tail -1 $OUT/gpu_tests_r2aq.log
cd /tmp
timeout -k 10 400 python3 -u $R/scripts/locate_sweep.py --rates 32 --backends task-ac,task,task-packed,task-ac-mid,task-mid --coop 0 --env "KFMI_SPLIT=1,4" > $OUT/locate_split_r2aq.jsonl 2> $OUT/locate_split_r2aq.log || { tail -30 $OUT/locate_split_r2aq.log; exit 32; }
timeout -k 10 500 python3 -u $R/scripts/locate_sweep.py --k 4 --rates 32 --backends task-grp --coop 0 --env "KFMI_SPLIT=1,4" >> $OUT/locate_split_r2aq.jsonl 2>> $OUT/locate_split_r2aq.log || { tail -30 $OUT/locate_split_r2aq.log; exit 33; }
cut -c1-230 $OUT/locate_split_r2aq.jsonl
