#!/bin/bash
# Round-1 session I: locate -- GPU tests, then the bench with the locate leg.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests/test_locate.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests_locate.log 2>&1 || { echo locate_tests_failed; tail -40 $OUT/gpu_tests_locate.log; exit 21; }
tail -2 $OUT/gpu_tests_locate.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_i.log 2>&1 || { echo tests_failed; tail -30 $OUT/gpu_tests_i.log; exit 22; }
tail -1 $OUT/gpu_tests_i.log
cd /tmp
timeout -k 10 500 python3 $R/bench.py > $OUT/bench_r01i.json 2> $OUT/bench_r01i.log || { tail -20 $OUT/bench_r01i.log; exit 33; }
python3 -c "import json; d=json.load(open('$OUT/bench_r01i.json')); print(d['value'], d['ms_per_step'], d['roofline']['lf_ms'], d['variants'].get('locate'))"
