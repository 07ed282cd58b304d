#!/bin/bash
# Round-4 session M: host <-> device copy rates (pageable direct, pinned, staged by chunk / buffers / threads)
# for the transfer entry points.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 300 k-step_fm-index_amd/bin/copy_probe 1.5 16 > $OUT/copy_probe_r4m.jsonl 2> $OUT/copy_probe_r4m.log || { tail -20 $OUT/copy_probe_r4m.log; exit 31; }
cat $OUT/copy_probe_r4m.jsonl
echo done
