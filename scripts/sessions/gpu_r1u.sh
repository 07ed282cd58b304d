#!/bin/bash
# Round-1 session U: refresh -- full GPU suite + smoke, default bench, bench at
# config #5's read length (150 bp, 10M per GPU), rocprof kernel stats of the
# default bench including every variant.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_u.log 2>&1 || { echo tests_failed; tail -40 $OUT/gpu_tests_u.log; exit 21; }
tail -1 $OUT/gpu_tests_u.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_u.log 2>&1 || { tail -20 $OUT/smoke_u.log; exit 22; }
tail -1 $OUT/smoke_u.log
cd /tmp
timeout -k 10 600 python3 $R/bench.py > $OUT/bench_r01u.json 2> $OUT/bench_r01u.log || { tail -20 $OUT/bench_r01u.log; exit 31; }
echo bench_done
timeout -k 10 600 python3 $R/bench.py --qlen 150 --variants task-mid,coop-mid,coop-ac128 --no-md5 --cpu-sample 1000000 > $OUT/bench_r01u_q150.json 2> $OUT/bench_r01u_q150.log || { tail -20 $OUT/bench_r01u_q150.log; exit 32; }
echo bench150_done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_r01u -o bench --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-sample 0 --e2e-steps 0 > $OUT/prof_bench_r01u.json 2> $OUT/prof_bench_r01u.log || exit 33
echo prof_done
