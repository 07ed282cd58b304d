#!/bin/bash
# Round-1 session C: bench (default backend task-mid) under rocprofv3 kernel
# trace, plus TCC request counters for the MID kernels.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 python3 $R/bench.py > $OUT/b_mid.json 2> $OUT/b_mid.log || exit 31
echo bench_done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_r1c -o bench --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --variants "" --cpu-sample 0 > $OUT/prof_mid.json 2> $OUT/prof_mid.log || exit 32
echo prof_done
SETS=("TCC_EA0_RDREQ_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_DRAM_sum"
      "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_LEVEL_sum TCC_REQ_sum")
i=0
for S in "${SETS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $S --kernel-include-regex "task_kernel|coop_kernel" -d $OUT/pmc_mid_$i -o p --output-format csv -- python3 $R/scripts/sweep.py --backends task-mid,coop-mid --steps 1 > $OUT/pmc_mid_$i.jsonl 2> $OUT/pmc_mid_$i.log || exit 33
  echo pmc_set_$i done
done
