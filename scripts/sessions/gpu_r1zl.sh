#!/bin/bash
# Round-1 session ZL (fresh container rebuild): GPU parity suite + smoke on the
# rebuilt tree, then the ZK profile refresh (default bench, rocprofv3 kernel
# stats, one TCC PMC pass).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests_r01zl.log 2>&1 || { tail -30 $OUT/gpu_tests_r01zl.log; exit 21; }
tail -3 $OUT/gpu_tests_r01zl.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke_r01zl.log 2>&1 || { tail -20 $OUT/smoke_r01zl.log; exit 22; }
tail -1 $OUT/smoke_r01zl.log
exec_zk=$R/scripts/gpu_r1zk.sh
bash $exec_zk
