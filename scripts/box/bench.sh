#!/bin/bash
# The driver's bench command on the box, plain and under rocprofv3 --kernel-trace --stats,
# then every row's rocprof kernel time (scripts/rows_from_trace.py):
#   bash scripts/box/bench.sh <tag> [--noprof]
set -o pipefail
T=${1:?tag}
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp KFMI_BENCH_LOGDIR=$OUT
cd /tmp
CMD="python3 $R/bench.py --gpus 1 --steps 20 --warmup 5"
timeout -k 10 600 $CMD --detail $OUT/bench_${T}_detail.json > $OUT/bench_$T.json 2> $OUT/bench_$T.err || { tail -20 $OUT/bench_$T.err; exit 35; }
wc -c $OUT/bench_$T.json $OUT/bench_$T.err
cut -c1-400 $OUT/bench_$T.json
[ "$2" = "--noprof" ] && exit 0
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d $OUT/prof_$T -o bench --output-format csv -- $CMD --detail $OUT/prof_bench_${T}_detail.json > $OUT/prof_bench_$T.json 2> $OUT/prof_bench_$T.err || { tail -20 $OUT/prof_bench_$T.err; exit 36; }
cut -c1-300 $OUT/prof_bench_$T.json
TR=$(find $OUT/prof_$T -name "*kernel_trace.csv" | head -1)
ST=$(find $OUT/prof_$T -name "*kernel_stats.csv" | head -1)
cp $TR $OUT/bench_${T}_kernel_trace.csv && cp $ST $OUT/bench_${T}_kernel_stats.csv
python3 $R/scripts/rows_from_trace.py --trace $TR --detail $OUT/prof_bench_${T}_detail.json > $OUT/rows_$T.json || exit 37
python3 $R/scripts/roofline_from_prof.py --trace $TR --bench $OUT/prof_bench_$T.json --warmup 5 --steps 20 > $OUT/roofline_$T.json || exit 38
cat $OUT/roofline_$T.json | head -20
