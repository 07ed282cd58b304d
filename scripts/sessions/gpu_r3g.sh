#!/bin/bash
# Round-3 session G: the driver's command profiled on the round-3 tree --
# plain, under rocprofv3 kernel trace + stats, and PMC passes of the LF kernel
# (fabric read requests with their queue level and DRAM credit stalls; L2
# hit/miss) -- plus the same request counters on gather_probe (3 GB table).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
CMD="python3 $R/bench.py --gpus 1 --steps 20 --warmup 5"
SHORT="python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --variants= --cpu-sample 0 --e2e-steps 0 --config5-queries 0 --no-kstep4 --ingest off --no-config1 --sa-rate 0 --parity-sample 0"
timeout -k 10 600 $CMD > $OUT/bench_r3g.json 2> $OUT/bench_r3g.log || { tail -20 $OUT/bench_r3g.log; exit 32; }
cut -c1-200 $OUT/bench_r3g.json
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d $OUT/prof_r3g -o bench --output-format csv -- $CMD > $OUT/prof_bench_r3g.json 2> $OUT/prof_bench_r3g.log || { tail -20 $OUT/prof_bench_r3g.log; exit 33; }
cut -c1-200 $OUT/prof_bench_r3g.json
timeout -s KILL 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_DRAM_sum GRBM_GUI_ACTIVE --kernel-include-regex "task_kernel" -d $OUT/pmc_r3g_a -o p --output-format csv -- $SHORT > $OUT/pmc_bench_r3g_a.json 2> $OUT/pmc_bench_r3g_a.log || { tail -20 $OUT/pmc_bench_r3g_a.log; exit 34; }
timeout -s KILL 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_GMI_CREDIT_STALL_sum TCC_EA0_RDREQ_IO_CREDIT_STALL_sum --kernel-include-regex "task_kernel" -d $OUT/pmc_r3g_b -o p --output-format csv -- $SHORT > $OUT/pmc_bench_r3g_b.json 2> $OUT/pmc_bench_r3g_b.log || { tail -20 $OUT/pmc_bench_r3g_b.log; exit 35; }
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_DRAM_sum GRBM_GUI_ACTIVE -d $OUT/pmc_r3g_probe -o p --output-format csv -- $R/k-step_fm-index_amd/bin/gather_probe 3 512 > $OUT/probe_r3g.jsonl 2> $OUT/probe_r3g.log || { tail -20 $OUT/probe_r3g.log; exit 36; }
ls $OUT/pmc_r3g_a $OUT/pmc_r3g_probe | head
