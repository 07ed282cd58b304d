#!/bin/bash
# Round-2 session BA: cooperative locate walk without the LDS line table (lane
# lines by shuffle: 32 KiB per workgroup, 5 per CU) -- locate tests, then rate
# 8 / 32 with KFMI_LOCATE_WG_PER_CU=4/5 on one box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_locate.py tests/test_groups.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r2ba.log 2>&1 || { tail -40 $OUT/gpu_tests_r2ba.log; exit 31; }
tail -2 $OUT/gpu_tests_r2ba.log
cd /tmp
timeout -k 10 600 python3 -u $R/scripts/locate_sweep.py --rates 8,32 --backends task-mid --coop 1 --env "KFMI_LOCATE_WG_PER_CU=4,5,4,5" > $OUT/locate_r2ba.jsonl 2> $OUT/locate_r2ba.log || { tail -30 $OUT/locate_r2ba.log; exit 32; }
python3 -c "
import json
for l in open('$OUT/locate_r2ba.jsonl'):
    d=json.loads(l); print(d['rate'], d['backend'], d['coop'], d['knobs'], d['kernel_ms'], d['pos_md5'][:8])
"
