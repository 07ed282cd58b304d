#!/bin/bash
# Round-4 session O: the driver's bench command with the trio per upload form (end_to_end.trio)
# and config #5 host-to-host on the default upload.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_r4o.json 2> $OUT/bench_r4o.log || { tail -20 $OUT/bench_r4o.log; exit 33; }
cat $OUT/bench_r4o.json
echo done
