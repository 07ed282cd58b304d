#!/bin/bash
# Round-2 session B: full GPU suite (incl. the 3 Gbase full-scale parity module
# and the group replication timing), then the default bench once.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
echo "affinity=$(python3 -c 'import os;print(len(os.sched_getaffinity(0)))') cpu_count=$(nproc --all) cpu.max=$(cat /sys/fs/cgroup/cpu.max 2>/dev/null)" > $OUT/r2b_host.txt
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r2b.log 2>&1 || { tail -40 $OUT/gpu_tests_r2b.log; exit 31; }
tail -3 $OUT/gpu_tests_r2b.log
cd /tmp
timeout -k 10 400 python3 $R/bench.py > $OUT/bench_r2b.json 2> $OUT/bench_r2b.log || { tail -30 $OUT/bench_r2b.log; exit 32; }
cut -c1-600 $OUT/bench_r2b.json
