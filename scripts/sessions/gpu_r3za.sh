#!/bin/bash
# Round-3 session ZA: what bounds the locate walk (rate 32, cooperative MID
# walk with the slot queue): fabric / L2 requests and instruction mix per
# launch, one PMC pass per counter set, plus the plain timing.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
LS="python3 $R/scripts/locate_sweep.py --rates 32 --backends task-mid --coop 1 --steps 3"
timeout -k 10 400 $LS > $OUT/locate_r3za.jsonl 2> $OUT/locate_r3za.log || { tail -20 $OUT/locate_r3za.log; exit 31; }
cut -c1-250 $OUT/locate_r3za.jsonl
timeout -s KILL 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum --kernel-include-regex "locate" -d $OUT/pmc_r3za_a -o p --output-format csv -- $LS > $OUT/pmc_r3za_a.jsonl 2> $OUT/pmc_r3za_a.log || { tail -20 $OUT/pmc_r3za_a.log; exit 32; }
timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU --kernel-include-regex "locate" -d $OUT/pmc_r3za_b -o p --output-format csv -- $LS > $OUT/pmc_r3za_b.jsonl 2> $OUT/pmc_r3za_b.log || { tail -20 $OUT/pmc_r3za_b.log; exit 33; }
echo done
