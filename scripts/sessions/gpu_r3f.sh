#!/bin/bash
# Round-3 session F: full GPU suite on the round-3 tree, smoke, the driver's
# bench command (N = 1) and an N = 2 rehearsal on the one card (expected to
# report n_gpus 1, shared_devices, no scaling claim; per-rank phases).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r3f.log 2>&1 || { tail -60 $OUT/gpu_tests_r3f.log; exit 31; }
tail -2 $OUT/gpu_tests_r3f.log
cd /tmp
timeout -k 10 600 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_r3f.json 2> $OUT/bench_r3f.log || { tail -30 $OUT/bench_r3f.log; exit 32; }
cut -c1-400 $OUT/bench_r3f.json
timeout -k 10 700 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 $R/bench.py --gpus 2 --steps 10 --warmup 5 --ref-size 1000000000 --queries 2000000 --config5-queries 2000000 > $OUT/bench_r3f_n2.json 2> $OUT/bench_r3f_n2.log || { tail -30 $OUT/bench_r3f_n2.log; exit 33; }
cut -c1-400 $OUT/bench_r3f_n2.json
