#!/bin/bash
# Round-4 session V: the final tree -- full GPU suite and smoke, --gpus 8 on the full config (eight
# self-spawned ranks on the one card: the N = 8 host side at full size), then the driver's N = 1 command.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r4v.log 2>&1 || { tail -60 $OUT/gpu_tests_r4v.log; exit 31; }
tail -2 $OUT/gpu_tests_r4v.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_r4v.log 2>&1 || { tail -30 $OUT/smoke_r4v.log; exit 32; }
cd /tmp
timeout -k 10 560 python3 $R/bench.py --gpus 8 --no-kstep4 --steps 10 --warmup 5 > $OUT/bench_r4v_n8full.json 2> $OUT/bench_r4v_n8full.log || { tail -30 $OUT/bench_r4v_n8full.log; exit 33; }
cut -c1-300 $OUT/bench_r4v_n8full.json
timeout -k 10 600 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_r4v.json 2> $OUT/bench_r4v.log || { tail -20 $OUT/bench_r4v.log; exit 34; }
cut -c1-300 $OUT/bench_r4v.json
echo done
