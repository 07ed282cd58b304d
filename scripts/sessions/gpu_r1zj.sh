#!/bin/bash
# Round-1 session ZJ: task-mid LF time vs device allocation order of the MID table
# (KFMI_ENT_FIRST=1: table allocated before the 4.5 GB staging buffer).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp
for mode in "0 0" "0 1" "1 0" "0 1" "0 0"; do
  set -- $mode
  KFMI_HOST_INTERLEAVE=$1 KFMI_ENT_FIRST=$2 timeout -k 10 300 python3 $R/bench.py --variants "" --no-config1 --cpu-sample 0 --e2e-steps 0 --sa-rate 0 --no-md5 > $OUT/ab_alloc.json 2> $OUT/ab_alloc.log || exit 31
  python3 -c "import json; d=json.load(open('$OUT/ab_alloc.json')); print('host_interleave=$1 ent_first=$2', d['value'], d['roofline']['lf_ms'], d['setup_s']['h2d'])"
done
