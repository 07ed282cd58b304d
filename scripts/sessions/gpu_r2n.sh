#!/bin/bash
# Round-2 session N: default bench (with the config #5 leg) at N=1, then the N=2 launch path on one GPU.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_r2n.json 2> $OUT/bench_r2n.log || { tail -30 $OUT/bench_r2n.log; exit 32; }
python3 -c "
import json; d=json.loads(open('$OUT/bench_r2n.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity'])
print(d['variants'].get('config5'))
"
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 $R/bench.py --gpus 2 --steps 10 --warmup 5 > $OUT/bench_r2n_n2.json 2> $OUT/bench_r2n_n2.log || { tail -30 $OUT/bench_r2n_n2.log; exit 33; }
python3 -c "
import json; d=json.loads(open('$OUT/bench_r2n_n2.json').read().strip().splitlines()[-1])
print(d['value'], d['n_gpus'], d['parity'], d['cpu_baseline']['value'])
print(d['variants'].get('config5'))
"
