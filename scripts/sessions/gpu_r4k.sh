#!/bin/bash
# Round-4 session K: request sizes and FETCH_SIZE (the guide's HBM recipe) for the headline LF kernel, with
# gather_probe's known line counts as the calibration (32/64/128-B lines, independent and chained).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
GP=$R/k-step_fm-index_amd/bin/gather_probe
SIZES="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
timeout -s KILL 120 rocprofv3 --pmc $SIZES -d $OUT/pmc_r4k_gp_sizes -o p --output-format csv -- $GP 3 512 > $OUT/pmc_r4k_gp_sizes.log 2>&1 || { tail -20 $OUT/pmc_r4k_gp_sizes.log; exit 31; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_r4k_gp_fetch -o p --output-format csv -- $GP 3 512 > $OUT/pmc_r4k_gp_fetch.log 2>&1 || { tail -20 $OUT/pmc_r4k_gp_fetch.log; exit 32; }
timeout -s KILL 300 rocprofv3 --pmc $SIZES --kernel-include-regex "task_kernel" -d $OUT/pmc_r4k_lf_sizes -o p --output-format csv -- python3 $R/scripts/pmc_variants.py --order $OUT/pmc_r4k_order_sizes.json --backends task-mid --k4-backends= > $OUT/pmc_r4k_lf_sizes.log 2>&1 || { tail -20 $OUT/pmc_r4k_lf_sizes.log; exit 33; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "task_kernel" -d $OUT/pmc_r4k_lf_fetch -o p --output-format csv -- python3 $R/scripts/pmc_variants.py --order $OUT/pmc_r4k_order_fetch.json --backends task-mid --k4-backends= > $OUT/pmc_r4k_lf_fetch.log 2>&1 || { tail -20 $OUT/pmc_r4k_lf_fetch.log; exit 34; }
for p in gp_sizes gp_fetch lf_sizes lf_fetch; do
  CSV=$(ls $OUT/pmc_r4k_$p/*/*counter_collection.csv $OUT/pmc_r4k_$p/*counter_collection.csv 2>/dev/null | sed -n 1p)
  cp $CSV $OUT/pmc_r4k_$p.csv || exit 35
  python3 $R/scripts/pmc_summary.py $OUT/pmc_r4k_$p.csv --skip-first > $OUT/pmc_r4k_$p.jsonl || exit 36
  cat $OUT/pmc_r4k_$p.jsonl
done
echo done
