#!/bin/bash
# Round-3 session ZB: locate walk slot-queue chunk size (KFMI_LOCATE_CHUNK) at
# SA rates 8 and 32 -- positions md5-compared across chunks -- then the locate
# GPU tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 500 python3 -u $R/scripts/locate_sweep.py --rates 8,32 --backends task-mid --coop 1 --steps 5 --env "KFMI_LOCATE_CHUNK=256,64,128,512,1024,256" > $OUT/locate_r3zb.jsonl 2> $OUT/locate_r3zb.log || { tail -20 $OUT/locate_r3zb.log; exit 31; }
cut -c1-230 $OUT/locate_r3zb.jsonl
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_locate.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/locate_tests_r3zb.log 2>&1 || { tail -40 $OUT/locate_tests_r3zb.log; exit 32; }
tail -2 $OUT/locate_tests_r3zb.log
