#!/bin/bash
# Round-3 session X: the final round-3 tree (coop counters in the DMA,
# pre-addressed rounds; 8 lanes per request on the grouped-counter lines) --
# full GPU suite, smoke, the K = 4 coop sweep, the driver's bench command,
# and the same command under rocprofv3 kernel trace + stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r3x.log 2>&1 || { tail -60 $OUT/gpu_tests_r3x.log; exit 31; }
tail -2 $OUT/gpu_tests_r3x.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_r3x.log 2>&1 || { tail -30 $OUT/smoke_r3x.log; exit 32; }
cd /tmp
timeout -k 10 600 python3 -u $R/scripts/sweep.py --k 4 --backends coop-grp,task-grp --env "KFMI_COOP_ISSUE=1,0" --steps 10 > $OUT/sweep_k4_r3x.jsonl 2> $OUT/sweep_k4_r3x.log || { tail -30 $OUT/sweep_k4_r3x.log; exit 33; }
cut -c1-170 $OUT/sweep_k4_r3x.jsonl
CMD="python3 $R/bench.py --gpus 1 --steps 20 --warmup 5"
timeout -k 10 600 $CMD > $OUT/bench_r3x.json 2> $OUT/bench_r3x.log || { tail -20 $OUT/bench_r3x.log; exit 34; }
cut -c1-300 $OUT/bench_r3x.json
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d $OUT/prof_r3x -o bench --output-format csv -- $CMD > $OUT/prof_bench_r3x.json 2> $OUT/prof_bench_r3x.log || { tail -20 $OUT/prof_bench_r3x.log; exit 35; }
cut -c1-200 $OUT/prof_bench_r3x.json
SHORT="python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --variants= --cpu-sample 0 --e2e-steps 0 --config5-queries 0 --no-kstep4 --ingest off --no-config1 --sa-rate 0 --parity-sample 0"
timeout -s KILL 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum --kernel-include-regex "task_kernel" -d $OUT/pmc_r3x -o p --output-format csv -- $SHORT > $OUT/pmc_bench_r3x.json 2> $OUT/pmc_bench_r3x.log || { tail -20 $OUT/pmc_bench_r3x.log; exit 36; }
echo done
