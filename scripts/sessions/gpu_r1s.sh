#!/bin/bash
# Round-1 session S: word skipping in the streaming LF (large d) -- GPU suite, d sweeps, locate.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_s.log 2>&1 || { echo tests_failed; tail -40 $OUT/gpu_tests_s.log; exit 21; }
tail -1 $OUT/gpu_tests_s.log
cd /tmp
ALL=task,coop,task-ac,coop-ac,task-packed,coop-packed,task-mid,coop-mid,task-ac128,coop-ac128
for D in 192 448; do
  timeout -k 10 500 python3 $R/scripts/sweep.py --k 2 --d $D --backends $ALL --steps 3 > $OUT/sweep_d${D}_s.jsonl 2> $OUT/sweep_d${D}_s.log || exit 31
done
timeout -k 10 500 python3 $R/scripts/locate_sweep.py --rates 32 --regs 0 --backends task-mid > $OUT/locate_sweep_s.jsonl 2> $OUT/locate_sweep_s.log || exit 32
cat $OUT/sweep_d192_s.jsonl $OUT/sweep_d448_s.jsonl $OUT/locate_sweep_s.jsonl | cut -c1-150
