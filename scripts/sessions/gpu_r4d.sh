#!/bin/bash
# Round-4 session D: N > 1 host readiness on the one-card box -- streamed-search host contention at
# P = 1, 2, 4, 8 ranks, the self-spawned --gpus 8 rehearsal (1 Gbase), and --gpus 2 on the full
# config #2 text (3 Gbase, ranks building in turn on the shared card).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 500 python3 -u $R/scripts/stream_contention.py --procs 1 2 4 8 --ref-size 300000000 --rounds 5 --out $OUT/stream_contention_r4d.jsonl > $OUT/stream_contention_r4d.log 2>&1 || { tail -30 $OUT/stream_contention_r4d.log; exit 31; }
tail -5 $OUT/stream_contention_r4d.log
timeout -k 10 400 python3 $R/bench.py --gpus 8 --ref-size 1000000000 --no-kstep4 --steps 10 --warmup 10 > $OUT/bench_r4d_n8.json 2> $OUT/bench_r4d_n8.log || { tail -30 $OUT/bench_r4d_n8.log; exit 32; }
cut -c1-300 $OUT/bench_r4d_n8.json
timeout -k 10 500 python3 $R/bench.py --gpus 2 --no-kstep4 --steps 20 --warmup 5 > $OUT/bench_r4d_n2full.json 2> $OUT/bench_r4d_n2full.log || { tail -30 $OUT/bench_r4d_n2full.log; exit 33; }
cut -c1-300 $OUT/bench_r4d_n2full.json
echo done
