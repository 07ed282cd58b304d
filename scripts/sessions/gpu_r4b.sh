#!/bin/bash
# Round-4 session B: the GPU suite after removing the neutral kernel forms, smoke, driver bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r4b.log 2>&1 || { tail -60 $OUT/gpu_tests_r4b.log; exit 31; }
tail -2 $OUT/gpu_tests_r4b.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_r4b.log 2>&1 || { tail -30 $OUT/smoke_r4b.log; exit 32; }
cd /tmp
timeout -k 10 600 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_r4b.json 2> $OUT/bench_r4b.log || { tail -20 $OUT/bench_r4b.log; exit 33; }
cut -c1-300 $OUT/bench_r4b.json
