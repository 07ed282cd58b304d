#!/bin/bash
# Round-3 session C: ref-alphabet GPU builder + searches on the reference's
# indexes of an hg38-style FASTA, streamed remainder reads, then the host
# contention sweep of the streamed search (1 and 2 concurrent processes).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_alphabet.py tests/test_stream.py tests/test_remainder.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r3c.log 2>&1 || { tail -60 $OUT/gpu_tests_r3c.log; exit 31; }
tail -2 $OUT/gpu_tests_r3c.log
timeout -k 10 600 python3 -u scripts/stream_contention.py --procs 1 2 --out $OUT/stream_contention_r3c.jsonl > $OUT/stream_contention_r3c.log 2>&1 || { tail -30 $OUT/stream_contention_r3c.log; exit 32; }
cat $OUT/stream_contention_r3c.log
