#!/bin/bash
# Round-2 session BI: device FASTA row kernel grid-stride (reads over 16 GB) --
# ingest, group and stream tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 500 python3 -u -m pytest tests/test_groups.py tests/test_ingest.py tests/test_stream.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r2bi.log 2>&1 || { tail -40 $OUT/gpu_tests_r2bi.log; exit 31; }
tail -2 $OUT/gpu_tests_r2bi.log
