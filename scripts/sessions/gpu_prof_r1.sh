#!/bin/bash
# Round-1 GPU session: builder tests, rocprofv3 kernel trace of the bench,
# variant sweep, counter list, FETCH_SIZE pass.  Stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python -m pytest tests/test_gpu_builder.py -m gpu -q > $OUT/t3.log 2>&1; rc=$?; echo builder_rc=$rc
[ $rc -le 1 ] || exit $rc
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_r1 -o bench --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --variants "" --cpu-sample 0 > $OUT/prof_bench.json 2> $OUT/prof_bench.log || exit 11
echo prof_done
timeout -k 10 400 python3 $R/scripts/sweep.py --backends task-packed,task,task-ac,coop,coop-ac,coop-packed --env "KFMI_QPT=1,2" --steps 5 > $OUT/sweep1.jsonl 2> $OUT/sweep1.log || exit 12
echo sweep_done
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "task_kernel|coop_kernel" -d $OUT/pmc_r1 -o fetch --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --variants "" --cpu-sample 0 > $OUT/pmc_bench.json 2> $OUT/pmc_bench.log || exit 13
echo pmc_done
