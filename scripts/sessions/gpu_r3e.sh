#!/bin/bash
# Round-3 session E: config #5's whole 80M x 150 bp batch on the 3 Gbase index
# (8-member device group on the card + streamed), and the alphabet GPU tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_fullscale.py -k config5_whole tests/test_alphabet.py -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r3e.log 2>&1 || { tail -60 $OUT/gpu_tests_r3e.log; exit 31; }
tail -5 $OUT/gpu_tests_r3e.log
