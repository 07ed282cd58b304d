#!/bin/bash
# Round-2 session AP: smoke(), default bench (K = 4 leg with task-grp), N = 2 rehearsal on the one card.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_r2ap.log 2>&1 || { tail -30 $OUT/smoke_r2ap.log; exit 30; }
tail -3 $OUT/smoke_r2ap.log
cd /tmp
timeout -k 10 600 python3 $R/bench.py > $OUT/bench_r2ap.json 2> $OUT/bench_r2ap.log || { tail -30 $OUT/bench_r2ap.log; exit 32; }
cut -c1-300 $OUT/bench_r2ap.json
timeout -k 10 700 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 $R/bench.py --gpus 2 --steps 10 --warmup 5 --ref-size 1000000000 --queries 2000000 --config5-queries 2000000 > $OUT/bench_r2ap_n2.json 2> $OUT/bench_r2ap_n2.log || { tail -30 $OUT/bench_r2ap_n2.log; exit 33; }
cut -c1-300 $OUT/bench_r2ap_n2.json
