#!/bin/bash
# Round-2 session L: do non-temporal deep-step loads (KFMI_NT_FROM) change the
# L2 hit count of task-mid?  One TCC pass over the sweep (order: none, 3, 4, 6, 8).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 600 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "task_kernel" -d $OUT/pmc_nt_r2l -o p --output-format csv -- python3 $R/scripts/sweep.py --backends task-mid --env "KFMI_NT_FROM=1000,3,4,6,8" --steps 4 > $OUT/pmc_nt_r2l.jsonl 2> $OUT/pmc_nt_r2l.log || { tail -20 $OUT/pmc_nt_r2l.log; exit 34; }
cat $OUT/pmc_nt_r2l.jsonl
python3 - <<PY
import csv, glob, collections
f = glob.glob("$OUT/pmc_nt_r2l/**/*counter_collection.csv", recursive=True)[0]
d = collections.defaultdict(dict)
for r in csv.DictReader(open(f)):
    if int(r["Grid_Size"]) == 10000128:
        d[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
        d[int(r["Dispatch_Id"])]["ms"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
ids = sorted(d)
for i, k in enumerate(ids):
    x = d[k]
    print(i, round(x["ms"], 3), int(x["TCC_EA0_RDREQ_sum"]) / 1e7, int(x["TCC_HIT_sum"]) / 1e7, int(x["TCC_MISS_sum"]) / 1e7)
PY
