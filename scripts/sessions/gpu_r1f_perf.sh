#!/bin/bash
# Round-1 session F: fused packing A/B (KFMI_FUSED=0/1) at 100 and 150 bp,
# then the default bench and its rocprofv3 kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 python3 $R/scripts/sweep.py --backends task-mid,task-ac,task --env "KFMI_FUSED=0,1" --steps 5 > $OUT/sweep_fused.jsonl 2> $OUT/sweep_fused.log || exit 31
echo fused100_done
timeout -k 10 400 python3 $R/scripts/sweep.py --backends task-mid --env "KFMI_FUSED=0,1" --qlen 150 --steps 5 > $OUT/sweep_fused_q150.jsonl 2> $OUT/sweep_fused_q150.log || exit 32
echo fused150_done
timeout -k 10 500 python3 $R/bench.py > $OUT/bench_r01f.json 2> $OUT/bench_r01f.log || exit 33
echo bench_done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_r01f -o bench --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --variants "" --cpu-sample 0 --e2e-steps 0 > $OUT/prof_bench_r01f.json 2> $OUT/prof_bench_r01f.log || exit 34
echo prof_done
