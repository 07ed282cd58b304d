#!/bin/bash
# Round-1 session ZI: A/B of the index upload path on one box (task-mid LF
# time): tag-100 entries interleaved on the device (default) vs on the host.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp
for mode in 0 1 0 1; do
  KFMI_HOST_INTERLEAVE=$mode timeout -k 10 300 python3 $R/bench.py --variants "" --no-config1 --cpu-sample 0 --e2e-steps 0 --sa-rate 0 --no-md5 > $OUT/ab_upload_$mode.json 2> $OUT/ab_upload_$mode.log || exit 31
  python3 -c "import json; d=json.load(open('$OUT/ab_upload_$mode.json')); print('host_interleave=$mode', d['value'], d['roofline']['lf_ms'], d['setup_s'])"
done
