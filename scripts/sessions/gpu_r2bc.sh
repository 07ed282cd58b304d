#!/bin/bash
# Round-2 session BC: can any load path beat the random-line request ceiling?
# coop 128-B gathers of a 3 GB table with sc0/sc1/nt cache-policy bits (raw
# buffer loads: bounds-checked; the first inline-asm version faulted), and the
# default probe on an uncached allocation.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
B=$R/k-step_fm-index_amd/bin/gather_probe
timeout -k 10 120 env PROBE_CPOL=1 $B 3 512 > $OUT/gather_cpol_r2bc.jsonl 2>&1 || { tail -20 $OUT/gather_cpol_r2bc.jsonl; exit 31; }
cat $OUT/gather_cpol_r2bc.jsonl
timeout -k 10 120 env PROBE_CPOL=1 PROBE_ALLOC=uncached $B 3 512 > $OUT/gather_uc_r2bc.jsonl 2>&1 || { tail -20 $OUT/gather_uc_r2bc.jsonl; exit 32; }
cat $OUT/gather_uc_r2bc.jsonl
