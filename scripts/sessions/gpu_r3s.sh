#!/bin/bash
# Round-3 session S: why the cooperative kernel trails the task kernel on the
# reference layouts (coop tag 101 / coop-ac tag 201 vs coop-mid and task-ac):
# fabric requests, instruction mix and wait cycles per LF launch, one PMC pass
# per counter set (3 Gbase, 10M x 100 bp, 3 timed launches per backend).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
SW="python3 $R/scripts/sweep.py --backends coop,coop-ac,coop-mid,task-ac --steps 3"
RX="coop_kernel|task_kernel"
timeout -s KILL 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum --kernel-include-regex "$RX" -d $OUT/pmc_r3s_a -o p --output-format csv -- $SW > $OUT/pmc_r3s_a.jsonl 2> $OUT/pmc_r3s_a.log || { tail -20 $OUT/pmc_r3s_a.log; exit 31; }
timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU --kernel-include-regex "$RX" -d $OUT/pmc_r3s_b -o p --output-format csv -- $SW > $OUT/pmc_r3s_b.jsonl 2> $OUT/pmc_r3s_b.log || { tail -20 $OUT/pmc_r3s_b.log; exit 32; }
timeout -s KILL 400 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT TCP_UTCL1_TRANSLATION_MISS_sum TCP_TCC_READ_REQ_sum --kernel-include-regex "$RX" -d $OUT/pmc_r3s_c -o p --output-format csv -- $SW > $OUT/pmc_r3s_c.jsonl 2> $OUT/pmc_r3s_c.log || { tail -20 $OUT/pmc_r3s_c.log; exit 33; }
find $OUT/pmc_r3s_a $OUT/pmc_r3s_b $OUT/pmc_r3s_c -name "*counter_collection.csv" | head
