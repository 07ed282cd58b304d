#!/bin/bash
# Round-4 session C: GPU suite after removing the neutral kernel forms, smoke, the driver's bench
# command (plain, then under rocprofv3 kernel trace + stats), and the per-backend PMC pass
# (scripts/pmc_variants.py) the bench's variant rows read.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r4c.log 2>&1 || { tail -60 $OUT/gpu_tests_r4c.log; exit 31; }
tail -2 $OUT/gpu_tests_r4c.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_r4c.log 2>&1 || { tail -30 $OUT/smoke_r4c.log; exit 32; }
cd /tmp
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_REQ_sum --kernel-include-regex "task_kernel|coop_kernel" -d $OUT/pmc_r4c -o p --output-format csv -- python3 $R/scripts/pmc_variants.py --order $OUT/pmc_r4c_order.json > $OUT/pmc_r4c.log 2>&1 || { tail -20 $OUT/pmc_r4c.log; exit 33; }
CSV=$(ls $OUT/pmc_r4c/*/*counter_collection.csv 2>/dev/null | head -1)
[ -z "$CSV" ] && CSV=$(find $OUT/pmc_r4c -name "*counter_collection.csv" | head -1)
mkdir -p $R/profiles/r04
python3 $R/scripts/traffic_variants.py $CSV $OUT/pmc_r4c_order.json --source "profiles/r04/pmc_r4c_variants.csv (rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_REQ_sum over scripts/pmc_variants.py, scripts/sessions/gpu_r4c.sh)" > $OUT/traffic_variants_r4c.json || exit 34
cp $OUT/traffic_variants_r4c.json $R/profiles/r04/traffic_variants.json
cp $CSV $OUT/pmc_r4c_variants.csv
CMD="python3 $R/bench.py --gpus 1 --steps 20 --warmup 5"
timeout -k 10 600 $CMD > $OUT/bench_r4c.json 2> $OUT/bench_r4c.log || { tail -20 $OUT/bench_r4c.log; exit 35; }
cut -c1-300 $OUT/bench_r4c.json
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d $OUT/prof_r4c -o bench --output-format csv -- $CMD > $OUT/prof_bench_r4c.json 2> $OUT/prof_bench_r4c.log || { tail -20 $OUT/prof_bench_r4c.log; exit 36; }
cut -c1-200 $OUT/prof_bench_r4c.json
echo done
