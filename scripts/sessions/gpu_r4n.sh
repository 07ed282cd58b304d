#!/bin/bash
# Round-4 session N: direct pageable h2d + host-packed query upload -- GPU suite, then the trio per upload form.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r4n.log 2>&1 || { tail -30 $OUT/gpu_tests_r4n.log; exit 31; }
tail -3 $OUT/gpu_tests_r4n.log
timeout -k 10 400 python3 scripts/upload_probe.py --reps 5 > $OUT/upload_probe_r4n.jsonl 2> $OUT/upload_probe_r4n.log || { tail -20 $OUT/upload_probe_r4n.log; exit 32; }
cat $OUT/upload_probe_r4n.jsonl
echo done
