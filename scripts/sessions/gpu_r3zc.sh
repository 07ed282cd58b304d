#!/bin/bash
# Round-3 session ZC: the tree as the round ends (locate chunk knob added) --
# full GPU suite, smoke, and an N = 2 rehearsal of the bench on the one card
# (reports 1 distinct GPU, no scaling claim).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r3zc.log 2>&1 || { tail -60 $OUT/gpu_tests_r3zc.log; exit 31; }
tail -2 $OUT/gpu_tests_r3zc.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_r3zc.log 2>&1 || { tail -30 $OUT/smoke_r3zc.log; exit 32; }
cd /tmp
timeout -k 10 700 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 $R/bench.py --gpus 2 --steps 10 --warmup 5 --ref-size 1000000000 --queries 2000000 --config5-queries 2000000 > $OUT/bench_r3zc_n2.json 2> $OUT/bench_r3zc_n2.log || { tail -30 $OUT/bench_r3zc_n2.log; exit 33; }
cut -c1-400 $OUT/bench_r3zc_n2.json
