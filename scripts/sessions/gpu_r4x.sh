#!/bin/bash
# Round-4 session X: the driver's bench command on the final tree (variant rows with traffic)
#
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_r4x.json 2> $OUT/bench_r4x.log || { tail -20 $OUT/bench_r4x.log; exit 33; }
cat $OUT/bench_r4x.json
echo done
