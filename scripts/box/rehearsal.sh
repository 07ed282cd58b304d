#!/bin/bash
# Multi-rank bench rehearsals on one card: N = 8 self-spawned and N = 2 under
# torch.distributed.run, K = 4 leg off (eight 96 GB tables do not fit one card); the line must
# stay <= 6 KB and stderr small.   bash scripts/box/rehearsal.sh <tag>
set -o pipefail
T=${1:?tag}
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 560 python3 $R/bench.py --gpus 8 --no-kstep4 --steps 10 --warmup 5 --detail $OUT/bench_${T}_n8_detail.json > $OUT/bench_${T}_n8.json 2> $OUT/bench_${T}_n8.err || { tail -30 $OUT/bench_${T}_n8.err; exit 41; }
wc -c $OUT/bench_${T}_n8.json $OUT/bench_${T}_n8.err
cut -c1-300 $OUT/bench_${T}_n8.json
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 $R/bench.py --gpus 2 --no-kstep4 --steps 10 --warmup 5 --detail $OUT/bench_${T}_n2_detail.json > $OUT/bench_${T}_n2.json 2> $OUT/bench_${T}_n2.err || { tail -30 $OUT/bench_${T}_n2.err; exit 42; }
wc -c $OUT/bench_${T}_n2.json $OUT/bench_${T}_n2.err
cut -c1-300 $OUT/bench_${T}_n2.json
