#!/bin/bash
# Round-3 session L: task kernels with the issue-all-then-wait fetch
# (fetch_ends_x4) -- parity (small geometries, alphabet fixtures, grid cap,
# streamed search, 3 Gbase md5 pins), then the backend sweep and the bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_alphabet.py tests/test_grid_cap.py tests/test_stream.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/l_parity.log 2>&1 || { tail -40 $OUT/l_parity.log; exit 31; }
tail -3 $OUT/l_parity.log
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_fullscale.py -m gpu -x -q -k "index_md5 or backend_full_scale" --timeout 600 --timeout-method thread > $OUT/l_full.log 2>&1 || { tail -40 $OUT/l_full.log; exit 32; }
tail -3 $OUT/l_full.log
cd /tmp
timeout -k 10 600 python3 -u $R/scripts/sweep.py --backends task,task-ac,task-mid,task-ac-mid,task-ac128,coop-mid --steps 10 > $OUT/sweep_r3l.jsonl 2> $OUT/sweep_r3l.log || { tail -30 $OUT/sweep_r3l.log; exit 33; }
cut -c1-200 $OUT/sweep_r3l.jsonl
cd $R
timeout -k 10 600 python3 -u bench.py > $OUT/bench_r3l.json 2> $OUT/bench_r3l.log || { tail -30 $OUT/bench_r3l.log; exit 34; }
cut -c1-400 $OUT/bench_r3l.json
