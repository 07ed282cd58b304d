#!/bin/bash
# Round-2 session AW: locate slot queue chosen by SA rate -- locate tests (incl.
# the forced queue / fixed order test), then rates 1 / 8 / 32 at the default.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_locate.py tests/test_groups.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r2aw.log 2>&1 || { tail -40 $OUT/gpu_tests_r2aw.log; exit 31; }
tail -2 $OUT/gpu_tests_r2aw.log
cd /tmp
timeout -k 10 600 python3 -u $R/scripts/locate_sweep.py --rates 1,8,32 --backends task-mid --coop 1,1 > $OUT/locate_r2aw.jsonl 2> $OUT/locate_r2aw.log || { tail -30 $OUT/locate_r2aw.log; exit 32; }
python3 -c "
import json
for l in open('$OUT/locate_r2aw.jsonl'):
    d=json.loads(l); print(d['rate'], d['backend'], d['coop'], d['knobs'], d['kernel_ms'], d['pos_md5'][:8])
"
