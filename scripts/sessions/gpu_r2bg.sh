#!/bin/bash
# Round-2 session BG: final full GPU suite, smoke(), default bench
# and N = 2 rehearsal on the round's final tree.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_r2bg.log 2>&1 || { tail -40 $OUT/gpu_tests_r2bg.log; exit 31; }
tail -2 $OUT/gpu_tests_r2bg.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_r2bg.log 2>&1 || { tail -30 $OUT/smoke_r2bg.log; exit 30; }
tail -2 $OUT/smoke_r2bg.log
cd /tmp
timeout -k 10 600 python3 $R/bench.py > $OUT/bench_r2bg.json 2> $OUT/bench_r2bg.log || { tail -30 $OUT/bench_r2bg.log; exit 32; }
cut -c1-300 $OUT/bench_r2bg.json
timeout -k 10 700 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 $R/bench.py --gpus 2 --steps 10 --warmup 5 --ref-size 1000000000 --queries 2000000 --config5-queries 2000000 > $OUT/bench_r2bg_n2.json 2> $OUT/bench_r2bg_n2.log || { tail -30 $OUT/bench_r2bg_n2.log; exit 33; }
cut -c1-300 $OUT/bench_r2bg_n2.json
