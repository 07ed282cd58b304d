#!/bin/bash
# Round-4 session E: the replay probe's modes (test + the driver's bench command, whose roofline carries
# them and the fixed gather-probe ceiling), then session D's N > 1 host-readiness runs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_probe.py tests/test_gpu_parity.py -k "probe or coop_backends" -x -q --timeout 250 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r4e.log 2>&1 || { tail -40 $OUT/gpu_tests_r4e.log; exit 31; }
tail -2 $OUT/gpu_tests_r4e.log
cd /tmp
timeout -k 10 600 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_r4e.json 2> $OUT/bench_r4e.log || { tail -20 $OUT/bench_r4e.log; exit 32; }
cut -c1-300 $OUT/bench_r4e.json
bash $R/scripts/sessions/gpu_r4d.sh
