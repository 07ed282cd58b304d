#!/bin/bash
# Round-2 session AV: slot queue in the cooperative locate walk only (scalar
# queue state), per-lane walk restored -- locate-related tests, then rate 8 / 32
# with KFMI_LOCATE_QUEUE=0/1 on one box (pos md5 must stay d1dc837d...).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_locate.py tests/test_groups.py tests/test_tools.py tests/test_kstep3.py tests/test_kstep4.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r2av.log 2>&1 || { tail -40 $OUT/gpu_tests_r2av.log; exit 31; }
tail -2 $OUT/gpu_tests_r2av.log
cd /tmp
timeout -k 10 600 python3 -u $R/scripts/locate_sweep.py --rates 1,8,32 --backends task-mid,task-ac --coop 0,1 --env "KFMI_LOCATE_QUEUE=0,1,0,1" > $OUT/locate_r2av.jsonl 2> $OUT/locate_r2av.log || { tail -30 $OUT/locate_r2av.log; exit 32; }
python3 -c "
import json
for l in open('$OUT/locate_r2av.jsonl'):
    d=json.loads(l); print(d['rate'], d['backend'], d['coop'], d['knobs'], d['kernel_ms'], d['pos_md5'][:8])
"
