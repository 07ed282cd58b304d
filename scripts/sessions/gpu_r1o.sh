#!/bin/bash
# Round-1 session O: default bench (reference CPU baseline leg) and the N=2
# launch path (torch.distributed.run, 2 ranks sharing the box's one GPU).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 python3 $R/bench.py > $OUT/bench_r01o.json 2> $OUT/bench_r01o.log || { tail -20 $OUT/bench_r01o.log; exit 31; }
python3 -c "import json; d=json.load(open('$OUT/bench_r01o.json')); print(d['value'], d['cpu_baseline'], d['variants'].get('cpu_port'))"
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 $R/bench.py --gpus 2 --steps 5 --warmup 2 > $OUT/bench_r01o_n2.json 2> $OUT/bench_r01o_n2.log || { tail -30 $OUT/bench_r01o_n2.log; exit 32; }
cat $OUT/bench_r01o_n2.json
