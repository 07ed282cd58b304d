#!/bin/bash
# Round-2 session X: full GPU suite, the default bench, an N=2 rehearsal (1 Gbase).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r2x.log 2>&1 || { tail -40 $OUT/gpu_tests_r2x.log; exit 31; }
tail -2 $OUT/gpu_tests_r2x.log
cd /tmp
timeout -k 10 600 python3 $R/bench.py > $OUT/bench_r2x.json 2> $OUT/bench_r2x.log || { tail -30 $OUT/bench_r2x.log; exit 32; }
cut -c1-300 $OUT/bench_r2x.json
timeout -k 10 700 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 $R/bench.py --gpus 2 --steps 10 --warmup 5 --ref-size 1000000000 --queries 2000000 --config5-queries 2000000 > $OUT/bench_r2x_n2.json 2> $OUT/bench_r2x_n2.log || { tail -30 $OUT/bench_r2x_n2.log; exit 33; }
cut -c1-300 $OUT/bench_r2x_n2.json
