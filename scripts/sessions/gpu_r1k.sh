#!/bin/bash
# Round-1 session K: bench + rocprofv3 kernel trace + TCC request counters of
# the fused task-mid LF kernel (profiles/r01, profiles/traffic.json).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 500 python3 $R/bench.py > $OUT/bench_r01k.json 2> $OUT/bench_r01k.log || { tail -20 $OUT/bench_r01k.log; exit 31; }
echo bench_done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_r01k -o bench --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --variants "" --cpu-sample 0 --e2e-steps 0 > $OUT/prof_bench_r01k.json 2> $OUT/prof_bench_r01k.log || exit 32
echo prof_done
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_DRAM_sum --kernel-include-regex "task_kernel|locate_kernel" -d $OUT/pmc_r01k_1 -o p --output-format csv -- python3 $R/scripts/sweep.py --backends task-mid --steps 1 > $OUT/pmc_r01k_1.jsonl 2> $OUT/pmc_r01k_1.log || exit 33
echo pmc1_done
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_EA0_RDREQ_LEVEL_sum --kernel-include-regex "task_kernel" -d $OUT/pmc_r01k_2 -o p --output-format csv -- python3 $R/scripts/sweep.py --backends task-mid --steps 1 > $OUT/pmc_r01k_2.jsonl 2> $OUT/pmc_r01k_2.log || exit 34
echo pmc2_done
