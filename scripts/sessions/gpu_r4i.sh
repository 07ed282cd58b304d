#!/bin/bash
# Round-4 session I: the final tree -- full GPU suite, smoke, the driver's bench command plain and under
# rocprofv3 kernel trace + stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r4i.log 2>&1 || { tail -60 $OUT/gpu_tests_r4i.log; exit 31; }
tail -2 $OUT/gpu_tests_r4i.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_r4i.log 2>&1 || { tail -30 $OUT/smoke_r4i.log; exit 32; }
cd /tmp
CMD="python3 $R/bench.py --gpus 1 --steps 20 --warmup 5"
timeout -k 10 600 $CMD > $OUT/bench_r4i.json 2> $OUT/bench_r4i.log || { tail -20 $OUT/bench_r4i.log; exit 33; }
cut -c1-300 $OUT/bench_r4i.json
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d $OUT/prof_r4i -o bench --output-format csv -- $CMD > $OUT/prof_bench_r4i.json 2> $OUT/prof_bench_r4i.log || { tail -20 $OUT/prof_bench_r4i.log; exit 34; }
cut -c1-200 $OUT/prof_bench_r4i.json
echo done
