#!/bin/bash
# Round-4 session Q: ASCII default upload through direct hipMemcpyAsync -- GPU suite, then the driver's bench
# command (trio per upload form, config #5 host-to-host).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r4q.log 2>&1 || { tail -30 $OUT/gpu_tests_r4q.log; exit 31; }
tail -2 $OUT/gpu_tests_r4q.log
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_r4q.json 2> $OUT/bench_r4q.log || { tail -20 $OUT/bench_r4q.log; exit 33; }
cat $OUT/bench_r4q.json
echo done
