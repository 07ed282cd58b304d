#!/bin/bash
# Round-2 session AI: split-issue gathers default on tables > 2 GB; full GPU suite incl. forced-split parity, bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 800 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r2ai.log 2>&1 || { tail -40 $OUT/gpu_tests_r2ai.log; exit 31; }
tail -2 $OUT/gpu_tests_r2ai.log
cd /tmp
timeout -k 10 600 python3 $R/bench.py > $OUT/bench_r2ai.json 2> $OUT/bench_r2ai.log || { tail -30 $OUT/bench_r2ai.log; exit 32; }
cut -c1-400 $OUT/bench_r2ai.json
