#!/bin/bash
# Round-2 session AX: full GPU suite (locate slot queue), smoke(), default bench
# (config #5 host-to-host wall), N = 2 rehearsal on the one card.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_r2ax.log 2>&1 || { tail -40 $OUT/gpu_tests_r2ax.log; exit 31; }
tail -2 $OUT/gpu_tests_r2ax.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_r2ax.log 2>&1 || { tail -30 $OUT/smoke_r2ax.log; exit 30; }
tail -2 $OUT/smoke_r2ax.log
cd /tmp
timeout -k 10 600 python3 $R/bench.py > $OUT/bench_r2ax.json 2> $OUT/bench_r2ax.log || { tail -30 $OUT/bench_r2ax.log; exit 32; }
cut -c1-300 $OUT/bench_r2ax.json
timeout -k 10 700 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 $R/bench.py --gpus 2 --steps 10 --warmup 5 --ref-size 1000000000 --queries 2000000 --config5-queries 2000000 > $OUT/bench_r2ax_n2.json 2> $OUT/bench_r2ax_n2.log || { tail -30 $OUT/bench_r2ax_n2.log; exit 33; }
cut -c1-300 $OUT/bench_r2ax_n2.json
