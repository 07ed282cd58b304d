#!/bin/bash
# Round-3 session A: changed paths -- streamed remainder reads, grid-stride
# loops under KFMI_MAX_GRID, device groups (breakdown test, guards), concurrent
# searches under the handle lock, exports; smoke; PMC counter list (is there a
# counter that separates Infinity-Cache hits?).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R

timeout -k 10 700 python3 -u -m pytest tests/test_grid_cap.py tests/test_groups.py tests/test_concurrent_search.py tests/test_host.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r3a.log 2>&1 || { tail -60 $OUT/gpu_tests_r3a.log; exit 31; }
tail -3 $OUT/gpu_tests_r3a.log
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_r3a.log 2>&1 || { tail -30 $OUT/smoke_r3a.log; exit 32; }
tail -2 $OUT/smoke_r3a.log
