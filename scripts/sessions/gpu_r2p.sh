#!/bin/bash
# Round-2 session P: default bench with the same-box request-ceiling probe.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_r2p.json 2> $OUT/bench_r2p.log || { tail -30 $OUT/bench_r2p.log; exit 32; }
python3 -c "
import json; d=json.loads(open('$OUT/bench_r2p.json').read().strip().splitlines()[-1])
r=d['roofline']; print(d['value'], d['ms_per_step'], r['frac'], r['line_requests_G_per_s'], r['line_request_ceiling_G_per_s'], r['line_request_frac'])
p=d['variants'].get('line_request_probe'); print({k:v for k,v in p.items() if k!='rows'} if p else None)
"
