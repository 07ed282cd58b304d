#!/bin/bash
# Round-2 session O: XCD-partition hypothesis -- reads laid out so that
# 256-read tile i holds suffix bucket i % B (round-robin workgroup dispatch ->
# each XCD's L2 sees 1/8 of the early-step intervals).  Timing, then TCC PMC.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 500 python3 -u $R/scripts/sweep.py --backends task-mid,coop-mid --sort-suffix 0 --xcd-tiles 8,16,4,7 --steps 10 > $OUT/sweep_xcd_r2o.jsonl 2> $OUT/sweep_xcd_r2o.log || { tail -30 $OUT/sweep_xcd_r2o.log; exit 32; }
cat $OUT/sweep_xcd_r2o.jsonl
timeout -s KILL 600 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "task_kernel" -d $OUT/pmc_xcd_r2o -o p --output-format csv -- python3 $R/scripts/sweep.py --backends task-mid --sort-suffix 0 --xcd-tiles 8 --steps 3 > $OUT/pmc_xcd_r2o.jsonl 2> $OUT/pmc_xcd_r2o.log || { tail -20 $OUT/pmc_xcd_r2o.log; exit 34; }
python3 - <<PY
import csv, glob, collections
f = glob.glob("$OUT/pmc_xcd_r2o/**/*counter_collection.csv", recursive=True)[0]
d = collections.defaultdict(dict)
for r in csv.DictReader(open(f)):
    if int(r["Grid_Size"]) == 10000128:
        d[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
        d[int(r["Dispatch_Id"])]["ms"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
for i, k in enumerate(sorted(d)):
    x = d[k]
    print(i, round(x["ms"], 3), int(x["TCC_EA0_RDREQ_sum"]) / 1e7, int(x["TCC_HIT_sum"]) / 1e7, int(x["TCC_MISS_sum"]) / 1e7)
PY
