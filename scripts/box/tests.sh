#!/bin/bash
# GPU suite + smoke on the box: bash scripts/box/tests.sh <tag>
set -o pipefail
T=${1:?tag}
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_$T.log 2>&1 || { tail -60 $OUT/gpu_tests_$T.log; exit 31; }
tail -2 $OUT/gpu_tests_$T.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$T.log 2>&1 || { tail -30 $OUT/smoke_$T.log; exit 32; }
tail -1 $OUT/smoke_$T.log
