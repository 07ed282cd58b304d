#!/bin/bash
# Round-2 session U: K=4 upload breakdown (kernel + memory-copy trace).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 python3 -u $R/scripts/k4_upload_probe.py > $OUT/k4_upload_r2u.txt 2>&1 || { tail -20 $OUT/k4_upload_r2u.txt; exit 31; }
cat $OUT/k4_upload_r2u.txt
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $OUT/prof_k4up_r2u -o p --output-format csv -- python3 $R/scripts/k4_upload_probe.py > $OUT/k4_upload_prof_r2u.txt 2>&1 || { tail -20 $OUT/k4_upload_prof_r2u.txt; exit 32; }
grep upload_s $OUT/k4_upload_prof_r2u.txt
for f in $(find $OUT/prof_k4up_r2u -name "*stats.csv"); do echo $f; head -15 $f | cut -c1-200; done
