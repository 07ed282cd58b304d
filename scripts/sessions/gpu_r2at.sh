#!/bin/bash
# Round-2 session AT: locate slot queue vs fixed slot order (KFMI_LOCATE_QUEUE=0/1)
# on one box, per-lane and cooperative walks, rate 8 / 32.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 python3 -u $R/scripts/locate_sweep.py --rates 8,32 --backends task-mid,task-ac --coop 0,1 --env "KFMI_LOCATE_QUEUE=0,1,0,1" > $OUT/locate_r2at.jsonl 2> $OUT/locate_r2at.log || { tail -30 $OUT/locate_r2at.log; exit 32; }
python3 -c "
import json
for l in open('$OUT/locate_r2at.jsonl'):
    d=json.loads(l); print(d['rate'], d['backend'], d['coop'], d['knobs'], d['kernel_ms'], d['pos_md5'][:8])
"
