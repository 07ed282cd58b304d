#!/bin/bash
# Round-3 session H: line-local previous-entry counting on the reference
# layouts (tag 101 task, tag 201 task-ac): parity (goldens incl. the AC
# sentinel text, random indexes at every d, AC tail blocks, B5, split gathers,
# alphabet indexes, 3 Gbase md5 pins) and the 3 Gbase sweep against task-mid.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_alphabet.py tests/test_remainder.py tests/test_locate.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r3h.log 2>&1 || { tail -60 $OUT/gpu_tests_r3h.log; exit 31; }
tail -2 $OUT/gpu_tests_r3h.log
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fullscale.py -k "full_scale and (task-ac or task-] or task-mid)" -m gpu -x -q --timeout 500 --timeout-method thread -p no:cacheprovider > $OUT/gpu_fullscale_r3h.log 2>&1 || { tail -60 $OUT/gpu_fullscale_r3h.log; exit 32; }
tail -2 $OUT/gpu_fullscale_r3h.log
cd /tmp
timeout -k 10 600 python3 -u $R/scripts/sweep.py --backends task-mid,task,task-ac,coop,coop-ac,task-mid --steps 10 > $OUT/sweep_r3h.jsonl 2> $OUT/sweep_r3h.log || { tail -30 $OUT/sweep_r3h.log; exit 33; }
cat $OUT/sweep_r3h.jsonl | cut -c1-250
