#!/bin/bash
# Round-3 session O: the asm fetch as the default task-kernel gather (form 7
# on split tables, 8 below) -- full GPU suite, the form sweep incl. the 6 GB
# AC128 table (four vs two groups), and the driver's bench command.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r3o.log 2>&1 || { tail -60 $OUT/gpu_tests_r3o.log; exit 31; }
tail -2 $OUT/gpu_tests_r3o.log
cd /tmp
timeout -k 10 600 python3 -u $R/scripts/sweep.py --backends task,task-ac,task-mid,task-ac-mid,task-packed --steps 10 > $OUT/sweep_r3o.jsonl 2> $OUT/sweep_r3o.log || { tail -30 $OUT/sweep_r3o.log; exit 33; }
cut -c1-170 $OUT/sweep_r3o.jsonl
timeout -k 10 600 python3 -u $R/scripts/sweep.py --backends task-ac128 --env "KFMI_SPLIT=4,6,7" --steps 10 > $OUT/sweep_ac128_r3o.jsonl 2> $OUT/sweep_ac128_r3o.log || { tail -30 $OUT/sweep_ac128_r3o.log; exit 34; }
cut -c1-170 $OUT/sweep_ac128_r3o.jsonl
timeout -k 10 600 python3 $R/bench.py > $OUT/bench_r3o.json 2> $OUT/bench_r3o.log || { tail -30 $OUT/bench_r3o.log; exit 35; }
cut -c1-300 $OUT/bench_r3o.json
