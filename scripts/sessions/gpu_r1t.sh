#!/bin/bash
# Round-1 session T: chunked streaming LF (large d) -- parity subset, d sweeps, locate.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_t.log 2>&1 || { echo tests_failed; tail -40 $OUT/gpu_tests_t.log; exit 21; }
tail -1 $OUT/gpu_tests_t.log
cd /tmp
for D in 192 448 960; do
  timeout -k 10 500 python3 $R/scripts/sweep.py --k 2 --d $D --backends task,task-ac,task-packed,task-mid --steps 3 > $OUT/sweep_d${D}_t.jsonl 2> $OUT/sweep_d${D}_t.log || exit 31
done
timeout -k 10 500 python3 $R/scripts/locate_sweep.py --rates 32 --regs 0 --backends task-mid > $OUT/locate_sweep_t.jsonl 2> $OUT/locate_sweep_t.log || exit 32
cat $OUT/sweep_d192_t.jsonl $OUT/sweep_d448_t.jsonl $OUT/sweep_d960_t.jsonl $OUT/locate_sweep_t.jsonl | cut -c1-110
