#!/bin/bash
# Round-1 session Q: ftab 16 bases (34 GB table), full GPU suite, default bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_q.log 2>&1 || { echo tests_failed; tail -40 $OUT/gpu_tests_q.log; exit 21; }
tail -1 $OUT/gpu_tests_q.log
cd /tmp
timeout -k 10 500 python3 $R/scripts/sweep.py --backends task-mid --env "KFMI_FTAB=14,16" --steps 10 > $OUT/sweep_ftab16.jsonl 2> $OUT/sweep_ftab16.log || exit 31
cat $OUT/sweep_ftab16.jsonl
timeout -k 10 600 python3 $R/bench.py > $OUT/bench_r01q.json 2> $OUT/bench_r01q.log || { tail -20 $OUT/bench_r01q.log; exit 32; }
python3 -c "import json; d=json.load(open('$OUT/bench_r01q.json')); print(d['value'], d['roofline']['frac'], d['cpu_baseline']['value'], {k: v.get('mqps') for k, v in d['variants'].items() if isinstance(v, dict)})"
