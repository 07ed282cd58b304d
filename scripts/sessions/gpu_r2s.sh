#!/bin/bash
# Round-2 session S: remainder table (m % K != 0) -- tests, then 150 bp / 151 bp
# reads on the 3 Gbase index at K=4 (coop-grp) and K=2 (task-mid).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_remainder.py tests/test_kstep4.py tests/test_ingest.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r2s.log 2>&1 || { tail -40 $OUT/gpu_tests_r2s.log; exit 31; }
tail -2 $OUT/gpu_tests_r2s.log
cd /tmp
timeout -k 10 400 python3 -u $R/scripts/sweep.py --k 4 --qlen 150 --backends coop-grp --steps 10 > $OUT/sweep_rem_r2s.jsonl 2> $OUT/sweep_rem_r2s.log || { tail -30 $OUT/sweep_rem_r2s.log; exit 32; }
timeout -k 10 400 python3 -u $R/scripts/sweep.py --k 2 --qlen 151 --backends task-mid,coop-mid --steps 10 >> $OUT/sweep_rem_r2s.jsonl 2>> $OUT/sweep_rem_r2s.log || { tail -30 $OUT/sweep_rem_r2s.log; exit 33; }
timeout -k 10 400 python3 -u $R/scripts/sweep.py --k 2 --qlen 150 --backends task-mid --steps 10 >> $OUT/sweep_rem_r2s.jsonl 2>> $OUT/sweep_rem_r2s.log || { tail -30 $OUT/sweep_rem_r2s.log; exit 34; }
cat $OUT/sweep_rem_r2s.jsonl
