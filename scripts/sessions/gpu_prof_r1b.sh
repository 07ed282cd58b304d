#!/bin/bash
# Round-1 session B: random-gather ceiling probe + TCC counters for the probe
# and the LF kernels (calibrates FETCH_SIZE / request sizes for this access
# pattern).  Stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 200 $R/k-step_fm-index_amd/bin/gather_probe 3 512 > $OUT/probe1.jsonl 2> $OUT/probe1.err || exit 21
echo probe_done
SETS=("TCC_EA0_RDREQ_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_DRAM_sum"
      "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_LEVEL_sum TCC_REQ_sum"
      "TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE SQ_WAVES_sum TA_BUSY_avr")
i=0
for S in "${SETS[@]}"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $S -d $OUT/pmc_probe_$i -o p --output-format csv -- $R/k-step_fm-index_amd/bin/gather_probe 3 256 > $OUT/pmc_probe_$i.log 2>&1 || exit 22
  timeout -k 10 300 rocprofv3 --pmc $S --kernel-include-regex "task_kernel|coop_kernel" -d $OUT/pmc_lf_$i -o p --output-format csv -- python3 $R/scripts/sweep.py --backends task-packed,task-ac,coop-ac,coop-packed,task --steps 1 > $OUT/pmc_lf_$i.jsonl 2> $OUT/pmc_lf_$i.log || exit 23
  echo pmc_set_$i done
done
