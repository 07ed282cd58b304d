#!/bin/bash
# Round-1 session ZB: host-packed streaming -- stream tests, then the e2e chunk
# sweep with host packing on and off.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python -u -m pytest tests/test_stream.py tests/test_qpack.py -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests_zb.log 2>&1 || { echo tests_failed; tail -40 $OUT/gpu_tests_zb.log; exit 21; }
tail -1 $OUT/gpu_tests_zb.log
cd /tmp
KFMI_STREAM_HOSTPACK=1 timeout -k 10 300 python3 $R/scripts/e2e_sweep.py --chunks 65536,131072,262144,524288,1048576 > $OUT/e2e_sweep_hostpack.jsonl 2> $OUT/e2e_sweep_hostpack.log || exit 31
cat $OUT/e2e_sweep_hostpack.jsonl
KFMI_STREAM_HOSTPACK=1 KFMI_HOST_THREADS=8 timeout -k 10 300 python3 $R/scripts/e2e_sweep.py --chunks 131072,262144,524288 > $OUT/e2e_sweep_hostpack_t8.jsonl 2> $OUT/e2e_sweep_hostpack_t8.log || exit 32
cat $OUT/e2e_sweep_hostpack_t8.jsonl
