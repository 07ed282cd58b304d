#!/bin/bash
# Round-4 session Z4: the driver's bench command on the final tree under rocprofv3 --kernel-trace --stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
CMD="python3 $R/bench.py --gpus 1 --steps 20 --warmup 5"
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d $OUT/prof_r4z4 -o bench --output-format csv -- $CMD > $OUT/prof_bench_r4z4.json 2> $OUT/prof_bench_r4z4.log || { tail -20 $OUT/prof_bench_r4z4.log; exit 34; }
cut -c1-200 $OUT/prof_bench_r4z4.json
echo done
