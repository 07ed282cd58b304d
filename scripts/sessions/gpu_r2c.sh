#!/bin/bash
# Round-2 session C: group tests, then the driver's exact bench command three
# times on one lease: plain, under rocprofv3 kernel trace + stats, and under one
# TCC PMC pass; roofline of the timed launches from the trace + PMC.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_groups.py -m gpu -x -q -s --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r2c.log 2>&1 || { tail -40 $OUT/gpu_tests_r2c.log; exit 31; }
tail -3 $OUT/gpu_tests_r2c.log
cd /tmp
CMD="python3 $R/bench.py --gpus 1 --steps 20 --warmup 5"
timeout -k 10 400 $CMD > $OUT/bench_r2c.json 2> $OUT/bench_r2c.log || { tail -30 $OUT/bench_r2c.log; exit 32; }
cut -c1-400 $OUT/bench_r2c.json
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof_r2c -o bench --output-format csv -- $CMD > $OUT/prof_bench_r2c.json 2> $OUT/prof_bench_r2c.log || { tail -20 $OUT/prof_bench_r2c.log; exit 33; }
echo prof_done
timeout -s KILL 600 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "task_kernel" -d $OUT/pmc_r2c -o p --output-format csv -- $CMD > $OUT/pmc_bench_r2c.json 2> $OUT/pmc_bench_r2c.log || { tail -20 $OUT/pmc_bench_r2c.log; exit 34; }
echo pmc_done
T=$(find $OUT/prof_r2c -name "*kernel_trace.csv" | head -1)
P=$(find $OUT/pmc_r2c -name "*counter_collection.csv" | head -1)
python3 $R/scripts/roofline_from_prof.py --trace $T --pmc $P --bench $OUT/prof_bench_r2c.json --warmup 5 --steps 20 > $OUT/roofline_r2c.json && cat $OUT/roofline_r2c.json
