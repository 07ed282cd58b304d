#!/bin/bash
# Round-3 session R: pre-addressed coop staging rounds (KFMI_COOP_ISSUE) --
# full GPU suite (incl. both issue forms forced), the coop sweep at K = 2 and
# K = 4 with the form swept, smoke, then the driver's bench command.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r3r.log 2>&1 || { tail -60 $OUT/gpu_tests_r3r.log; exit 31; }
tail -2 $OUT/gpu_tests_r3r.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_r3r.log 2>&1 || { tail -30 $OUT/smoke_r3r.log; exit 32; }
cd /tmp
timeout -k 10 600 python3 -u $R/scripts/sweep.py --backends coop,coop-ac,coop-mid,coop-ac128,coop-ac-mid --env "KFMI_COOP_ISSUE=0,1" --steps 10 > $OUT/sweep_r3r.jsonl 2> $OUT/sweep_r3r.log || { tail -30 $OUT/sweep_r3r.log; exit 33; }
cut -c1-170 $OUT/sweep_r3r.jsonl
timeout -k 10 600 python3 -u $R/scripts/sweep.py --k 4 --backends coop-grp,task-grp --env "KFMI_COOP_ISSUE=0,1" --steps 10 > $OUT/sweep_k4_r3r.jsonl 2> $OUT/sweep_k4_r3r.log || { tail -30 $OUT/sweep_k4_r3r.log; exit 34; }
cut -c1-170 $OUT/sweep_k4_r3r.jsonl
timeout -k 10 600 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_r3r.json 2> $OUT/bench_r3r.log || { tail -20 $OUT/bench_r3r.log; exit 35; }
cut -c1-300 $OUT/bench_r3r.json
