#!/bin/bash
# Round-4 session U: streamed search chunk ramp -- stream GPU tests, then pinned / pageable host-to-host with
# the ramp off and on (separate processes, adaptive and always-pack modes).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_stream.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r4u.log 2>&1 || { tail -30 $OUT/gpu_tests_r4u.log; exit 31; }
tail -2 $OUT/gpu_tests_r4u.log
: > $OUT/e2e_ramp_r4u.jsonl
for rp in 0 1 0 1; do
  KFMI_STREAM_RAMP=$rp E2E_ISA=avx512 E2E_MODES=2,1 timeout -k 10 400 python3 scripts/e2e_modes.py > $OUT/e2e_ramp_r4u_$rp.tmp 2>> $OUT/e2e_ramp_r4u.log || { tail -20 $OUT/e2e_ramp_r4u.log; exit 32; }
  sed "s/^{/{\"ramp\": $rp, /" $OUT/e2e_ramp_r4u_$rp.tmp >> $OUT/e2e_ramp_r4u.jsonl
done
rm -f $OUT/e2e_ramp_r4u_*.tmp
cat $OUT/e2e_ramp_r4u.jsonl
echo done
