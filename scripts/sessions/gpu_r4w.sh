#!/bin/bash
# Round-4 session W: the streamed search's chunk ramp interleaved call by call with equal chunks in one
# process (9 rounds), adaptive and always-pack, pinned and pageable; the stream GPU tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_stream.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r4w.log 2>&1 || { tail -30 $OUT/gpu_tests_r4w.log; exit 31; }
tail -1 $OUT/gpu_tests_r4w.log
E2E_ISA=avx512 E2E_MODES=2,2r,1,1r E2E_ROUNDS=9 timeout -k 10 500 python3 scripts/e2e_modes.py > $OUT/e2e_ramp_r4w.jsonl 2> $OUT/e2e_ramp_r4w.log || { tail -20 $OUT/e2e_ramp_r4w.log; exit 32; }
cat $OUT/e2e_ramp_r4w.jsonl
echo done
