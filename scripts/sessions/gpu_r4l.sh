#!/bin/bash
# Round-4 session L: the driver's bench command with roofline.traffic from the FETCH_SIZE pass and the
# ceiling as max(probe, replay with PMC-counted requests).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_r4l.json 2> $OUT/bench_r4l.log || { tail -20 $OUT/bench_r4l.log; exit 33; }
cat $OUT/bench_r4l.json
echo done
