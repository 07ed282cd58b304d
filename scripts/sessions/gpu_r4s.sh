#!/bin/bash
# Round-4 session S: streamed search with pageable ASCII chunks copied by the runtime (KFMI_STREAM_DIRECT)
# against the workers' staging copy, ASCII-only and adaptive, pinned and pageable input.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
E2E_ISA=avx512 E2E_MODES=0,0d,2,2d,1 timeout -k 10 600 python3 scripts/e2e_modes.py > $OUT/e2e_direct_r4s.jsonl 2> $OUT/e2e_direct_r4s.log || { tail -20 $OUT/e2e_direct_r4s.log; exit 31; }
cat $OUT/e2e_direct_r4s.jsonl
echo done
