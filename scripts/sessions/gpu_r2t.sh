#!/bin/bash
# Round-2 session T: device-resident index (no host image) tests, then the
# default bench (K=4 leg now built without a host image, on every rank).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_device_resident.py tests/test_gpu_builder.py tests/test_kstep4.py tests/test_groups.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r2t.log 2>&1 || { tail -40 $OUT/gpu_tests_r2t.log; exit 31; }
tail -2 $OUT/gpu_tests_r2t.log
cd /tmp
timeout -k 10 600 python3 $R/bench.py > $OUT/bench_r2t.json 2> $OUT/bench_r2t.log || { tail -30 $OUT/bench_r2t.log; exit 32; }
cut -c1-300 $OUT/bench_r2t.json
grep -n "K=4 leg" $OUT/bench_r2t.log | cut -c1-900
