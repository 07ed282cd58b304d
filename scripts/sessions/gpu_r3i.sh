#!/bin/bash
# Round-3 session I: line requests per read of the reference-layout task kernels
# with line-local counting, split-issue 1 vs 4 (PMC TCC_EA0_RDREQ per launch).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 python3 -u $R/scripts/sweep.py --backends task,task-ac --env "KFMI_SPLIT=1,4" --steps 10 > $OUT/sweep_r3i.jsonl 2> $OUT/sweep_r3i.log || { tail -30 $OUT/sweep_r3i.log; exit 33; }
cut -c1-200 $OUT/sweep_r3i.jsonl
timeout -s KILL 600 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "task_kernel" -d $OUT/pmc_r3i -o p --output-format csv -- python3 $R/scripts/sweep.py --backends task,task-ac,task-mid --steps 2 > $OUT/pmc_sweep_r3i.jsonl 2> $OUT/pmc_sweep_r3i.log || { tail -20 $OUT/pmc_sweep_r3i.log; exit 34; }
ls $OUT/pmc_r3i
