#!/bin/bash
# Round-1 session X: full GPU suite + default bench (config #1 leg, CPU model, 1-thread rate).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_x.log 2>&1 || { echo tests_failed; tail -40 $OUT/gpu_tests_x.log; exit 21; }
tail -1 $OUT/gpu_tests_x.log
cd /tmp
timeout -k 10 700 python3 $R/bench.py > $OUT/bench_r01x.json 2> $OUT/bench_r01x.log || { tail -20 $OUT/bench_r01x.log; exit 31; }
python3 -c "import json; d=json.load(open('$OUT/bench_r01x.json')); v=d['variants']; print(d['value'], d['roofline']['achieved'], d['roofline']['frac'], d['cpu_baseline']['value'], d['cpu_baseline']['cpu_model'], v.get('cpu_port_1thread'), v.get('config1_64mbase'), v['coop-mid'])"
