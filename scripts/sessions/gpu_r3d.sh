#!/bin/bash
# Round-3 session D: (1) host contention sweep of the streamed search, 7 rounds
# (round 0 = warm-up, excluded); (2) N = 2 rehearsal at the FULL config (3 Gbase,
# 10M reads per rank) on the one card -- per-rank phase wall times for the
# N = 8 projection; the two K = 4 indexes (~150 GB build peak each) may not
# both fit one card: the leg must then report the failing rank's error
# without hanging the other (Steps / all_ok).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 700 python3 -u scripts/stream_contention.py --procs 1 2 --out $OUT/stream_contention_r3d.jsonl > $OUT/stream_contention_r3d.log 2>&1 || { tail -30 $OUT/stream_contention_r3d.log; exit 32; }
cat $OUT/stream_contention_r3d.log
cd /tmp
timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 $R/bench.py --gpus 2 --steps 20 --warmup 5 > $OUT/bench_r3d_n2full.json 2> $OUT/bench_r3d_n2full.log || { tail -30 $OUT/bench_r3d_n2full.log; exit 33; }
cut -c1-300 $OUT/bench_r3d_n2full.json
