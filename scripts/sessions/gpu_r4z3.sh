#!/bin/bash
# Round-4 session Z3: the final tree after the host builder buffers on 2 MB pages -- full GPU suite, smoke, the driver's
# bench command.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r4z3.log 2>&1 || { tail -60 $OUT/gpu_tests_r4z3.log; exit 31; }
tail -2 $OUT/gpu_tests_r4z3.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_r4z3.log 2>&1 || { tail -30 $OUT/smoke_r4z3.log; exit 32; }
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_r4z3.json 2> $OUT/bench_r4z3.log || { tail -20 $OUT/bench_r4z3.log; exit 33; }
cut -c1-300 $OUT/bench_r4z3.json
echo done
