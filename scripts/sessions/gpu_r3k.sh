#!/bin/bash
# Round-3 session K: cooperative kernel on the reference layouts (tag 101/201)
# with planes-only staging + line-local counting -- parity (small geometries,
# alphabet fixtures, 3 Gbase md5 pins), then the split / backend sweep.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_alphabet.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/k_parity.log 2>&1 || { tail -40 $OUT/k_parity.log; exit 31; }
tail -3 $OUT/k_parity.log
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_fullscale.py -m gpu -x -q -k "index_md5 or backend_full_scale" --timeout 600 --timeout-method thread > $OUT/k_full.log 2>&1 || { tail -40 $OUT/k_full.log; exit 32; }
tail -3 $OUT/k_full.log
cd /tmp
timeout -k 10 600 python3 -u $R/scripts/sweep.py --backends coop,coop-ac,task,task-ac --env "KFMI_SPLIT=1,4" --steps 10 > $OUT/sweep_r3k.jsonl 2> $OUT/sweep_r3k.log || { tail -30 $OUT/sweep_r3k.log; exit 33; }
cut -c1-200 $OUT/sweep_r3k.jsonl
