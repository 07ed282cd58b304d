#!/bin/bash
# Round-2 session BE (final tree of the round): the driver's exact bench command three times on one
# lease -- plain, under rocprofv3 kernel trace + stats, under one TCC PMC pass --
# and the roofline of the timed launches from the trace + PMC.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
CMD="python3 $R/bench.py --gpus 1 --steps 20 --warmup 5"
timeout -k 10 500 $CMD > $OUT/bench_r2be.json 2> $OUT/bench_r2be.log || { tail -30 $OUT/bench_r2be.log; exit 32; }
cut -c1-300 $OUT/bench_r2be.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_r2be -o bench --output-format csv -- $CMD > $OUT/prof_bench_r2be.json 2> $OUT/prof_bench_r2be.log || { tail -20 $OUT/prof_bench_r2be.log; exit 33; }
echo prof_done
timeout -s KILL 700 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "task_kernel" -d $OUT/pmc_r2be -o p --output-format csv -- $CMD > $OUT/pmc_bench_r2be.json 2> $OUT/pmc_bench_r2be.log || { tail -20 $OUT/pmc_bench_r2be.log; exit 34; }
echo pmc_done
T=$(find $OUT/prof_r2be -name "*kernel_trace.csv" | head -1)
P=$(find $OUT/pmc_r2be -name "*counter_collection.csv" | head -1)
python3 $R/scripts/roofline_from_prof.py --trace $T --pmc $P --bench $OUT/prof_bench_r2be.json --warmup 5 --steps 20 > $OUT/roofline_r2be.json && cat $OUT/roofline_r2be.json
