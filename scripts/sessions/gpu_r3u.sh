#!/bin/bash
# Round-3 session U: coop on the reference layouts with the counter chunk in
# the DMA for ends not counted from block b-1 (per-lane counter loads only
# for those) -- coop parity, the coop sweep, and the LF launch counters.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_alphabet.py tests/test_gpu_fullscale.py -m gpu -x -q -k "coop or index_md5" --timeout 600 --timeout-method thread -p no:cacheprovider > $OUT/u_parity.log 2>&1 || { tail -40 $OUT/u_parity.log; exit 31; }
tail -2 $OUT/u_parity.log
cd /tmp
timeout -k 10 600 python3 -u $R/scripts/sweep.py --backends coop,coop-ac,coop-mid,task-ac --env "KFMI_COOP_ISSUE=1,0" --steps 10 > $OUT/sweep_r3u.jsonl 2> $OUT/sweep_r3u.log || { tail -30 $OUT/sweep_r3u.log; exit 33; }
cut -c1-170 $OUT/sweep_r3u.jsonl
timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU --kernel-include-regex "coop_kernel|task_kernel" -d $OUT/pmc_r3u_b -o p --output-format csv -- python3 $R/scripts/sweep.py --backends coop,coop-ac,coop-mid,task-ac --steps 3 > $OUT/pmc_r3u_b.jsonl 2> $OUT/pmc_r3u_b.log || { tail -20 $OUT/pmc_r3u_b.log; exit 34; }
timeout -s KILL 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum --kernel-include-regex "coop_kernel|task_kernel" -d $OUT/pmc_r3u_a -o p --output-format csv -- python3 $R/scripts/sweep.py --backends coop,coop-ac,coop-mid,task-ac --steps 3 > $OUT/pmc_r3u_a.jsonl 2> $OUT/pmc_r3u_a.log || { tail -20 $OUT/pmc_r3u_a.log; exit 35; }
echo done
