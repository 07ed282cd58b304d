#!/bin/bash
# Round-1 session ZM: the N=2 launch path on the final tree (torch.distributed.run,
# 2 ranks sharing the box's one GPU), default bench arguments.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 $R/bench.py --gpus 2 > $OUT/bench_r01zm_n2.json 2> $OUT/bench_r01zm_n2.log || { tail -30 $OUT/bench_r01zm_n2.log; exit 32; }
cat $OUT/bench_r01zm_n2.json | cut -c1-400
