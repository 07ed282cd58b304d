#!/bin/bash
# Round-2 session H: parity module (incl. the AltCounters-on-MID128 backends and
# their tail blocks), stream tests, then 3 Gbase timings: ac-mid vs the AC
# backends, and the streamed-search mode x ISA sweep.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_stream.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r2h.log 2>&1 || { tail -40 $OUT/gpu_tests_r2h.log; exit 31; }
tail -2 $OUT/gpu_tests_r2h.log
cd /tmp
timeout -k 10 400 python3 -u $R/scripts/sweep.py --backends task-mid,task-ac-mid,coop-ac-mid,task-ac,coop-ac128 --steps 10 > $OUT/sweep_acmid_r2h.jsonl 2> $OUT/sweep_acmid_r2h.log || { tail -30 $OUT/sweep_acmid_r2h.log; exit 32; }
cat $OUT/sweep_acmid_r2h.jsonl
timeout -k 10 400 python3 -u $R/scripts/e2e_modes.py > $OUT/e2e_modes_r2h.jsonl 2> $OUT/e2e_modes_r2h.log || { tail -30 $OUT/e2e_modes_r2h.log; exit 33; }
cat $OUT/e2e_modes_r2h.jsonl
