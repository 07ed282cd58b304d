#!/bin/bash
# Round-2 session F: the N=2 launch path (torch.distributed.run, two ranks
# sharing the box's one GPU) with the per-rank parity / ingest / CPU baseline.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 $R/bench.py --gpus 2 --steps 10 --warmup 5 > $OUT/bench_r2f_n2.json 2> $OUT/bench_r2f_n2.log || { tail -30 $OUT/bench_r2f_n2.log; exit 32; }
python3 -c "
import json; d=json.loads(open('$OUT/bench_r2f_n2.json').read().strip().splitlines()[-1])
print(d['value'], d['n_gpus'], d['parity'], d['cpu_baseline']['value'], d['cpu_baseline']['cores'])
print({k: v for k, v in d['ranks'].items() if k != 'ranks'})
for r in d['ranks']['ranks']: print(r)
"
