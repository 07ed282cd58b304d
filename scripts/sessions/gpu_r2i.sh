#!/bin/bash
# Round-2 session I: parity module again (ac-mid tail rewrite), then 3 Gbase
# timings of the AltCounters-semantics backends.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r2i.log 2>&1 || { tail -40 $OUT/gpu_tests_r2i.log; exit 31; }
tail -2 $OUT/gpu_tests_r2i.log
cd /tmp
timeout -k 10 400 python3 -u $R/scripts/sweep.py --backends task-mid,task-ac-mid,coop-ac-mid,coop-mid,task-ac,coop-ac128 --steps 10 > $OUT/sweep_acmid_r2i.jsonl 2> $OUT/sweep_acmid_r2i.log || { tail -30 $OUT/sweep_acmid_r2i.log; exit 32; }
cat $OUT/sweep_acmid_r2i.jsonl
