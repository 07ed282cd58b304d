#!/bin/bash
# Round-2 session AU: per-lane locate walk A/B on one box -- round-1 kernel
# (fixed order, per-lane exit), queue + wave-uniform loop, queue + per-lane
# exit; cooperative walk with the queue beside them.  Rate 8 / 32.  (The
# KFMI_LOCATE_VAR variants were removed after this run: round-1 kernel kept.)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 python3 -u $R/scripts/locate_sweep.py --rates 8,32 --backends task-mid,task-ac --coop 0 --env "KFMI_LOCATE_VAR=old,ballot,brk,old,ballot,brk" > $OUT/locate_r2au.jsonl 2> $OUT/locate_r2au.log || { tail -30 $OUT/locate_r2au.log; exit 32; }
timeout -k 10 300 python3 -u $R/scripts/locate_sweep.py --rates 32 --backends task-mid --coop 1 --env "KFMI_LOCATE_QUEUE=0,1,0,1" >> $OUT/locate_r2au.jsonl 2>> $OUT/locate_r2au.log || { tail -30 $OUT/locate_r2au.log; exit 33; }
python3 -c "
import json
for l in open('$OUT/locate_r2au.jsonl'):
    d=json.loads(l); print(d['rate'], d['backend'], d['coop'], d['knobs'], d['kernel_ms'], d['pos_md5'][:8])
"
