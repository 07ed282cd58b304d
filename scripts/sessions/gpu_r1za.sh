#!/bin/bash
# Round-1 session ZA: kernel instantiations split over per-(K, layout) units --
# full GPU suite + smoke + default bench (same kernels, must match r01q/r01x).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_za.log 2>&1 || { echo tests_failed; tail -40 $OUT/gpu_tests_za.log; exit 21; }
tail -1 $OUT/gpu_tests_za.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_za.log 2>&1 || { tail -20 $OUT/smoke_za.log; exit 22; }
tail -1 $OUT/smoke_za.log
cd /tmp
timeout -k 10 700 python3 $R/bench.py > $OUT/bench_r01za.json 2> $OUT/bench_r01za.log || { tail -20 $OUT/bench_r01za.log; exit 31; }
python3 -c "import json; d=json.load(open('$OUT/bench_r01za.json')); v=d['variants']; print(d['value'], d['roofline']['achieved'], d['roofline']['frac'], d['cpu_baseline']['value'], v.get('config1_64mbase'), {k: (x.get('mqps') if isinstance(x, dict) else x) for k, x in v.items()})"
