#!/bin/bash
# Round-4 session F: the streamed search's cost model with the contended-link estimate -- its GPU
# tests, host contention at P = 1, 2, 4, 8 again, and --gpus 8 on the full config #2 text (3 Gbase,
# eight ranks on the one card: the N = 8 host side at full size).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_stream.py tests/test_groups.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r4f.log 2>&1 || { tail -40 $OUT/gpu_tests_r4f.log; exit 31; }
tail -2 $OUT/gpu_tests_r4f.log
cd /tmp
timeout -k 10 500 python3 -u $R/scripts/stream_contention.py --procs 1 2 4 8 --ref-size 300000000 --rounds 5 --out $OUT/stream_contention_r4f.jsonl > $OUT/stream_contention_r4f.log 2>&1 || { tail -30 $OUT/stream_contention_r4f.log; exit 32; }
tail -8 $OUT/stream_contention_r4f.log | cut -c1-200
timeout -k 10 560 python3 $R/bench.py --gpus 8 --no-kstep4 --steps 10 --warmup 5 > $OUT/bench_r4f_n8full.json 2> $OUT/bench_r4f_n8full.log || { tail -30 $OUT/bench_r4f_n8full.log; exit 33; }
cut -c1-300 $OUT/bench_r4f_n8full.json
echo done
