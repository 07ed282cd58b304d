#!/bin/bash
# Round-4 session J: fabric requests of the replay probe's kernels beside the LF kernel's (PMC), so the
# replay's request rate is measured, not estimated; then the driver's bench command (Infinity-Cache probe
# taken twice, best run per kind).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_REQ_sum --kernel-include-regex "task_kernel|replay_lines_kernel|replay_fetch_kernel" -d $OUT/pmc_r4j -o p --output-format csv -- python3 $R/scripts/pmc_replay.py > $OUT/pmc_r4j.log 2>&1 || { tail -20 $OUT/pmc_r4j.log; exit 31; }
CSV=$(find $OUT/pmc_r4j -name "*counter_collection.csv" | head -1)
cp $CSV $OUT/pmc_r4j_replay.csv
python3 $R/scripts/pmc_replay.py --summarize $CSV > $OUT/pmc_r4j_summary.jsonl || exit 32
cat $OUT/pmc_r4j_summary.jsonl
cd $R
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_r4j.json 2> $OUT/bench_r4j.log || { tail -20 $OUT/bench_r4j.log; exit 33; }
cat $OUT/bench_r4j.json
echo done
