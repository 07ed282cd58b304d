#!/bin/bash
# Round-2 session R: full GPU suite (incl. K=4), the default bench (with the
# K=4 coop-grp leg), then one TCC PMC pass of the K=4 sweep (lines per query).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r2r.log 2>&1 || { tail -40 $OUT/gpu_tests_r2r.log; exit 31; }
tail -2 $OUT/gpu_tests_r2r.log
cd /tmp
timeout -k 10 500 python3 $R/bench.py > $OUT/bench_r2r.json 2> $OUT/bench_r2r.log || { tail -30 $OUT/bench_r2r.log; exit 32; }
cut -c1-300 $OUT/bench_r2r.json
grep -n "K=4 leg" $OUT/bench_r2r.log | cut -c1-600
timeout -s KILL 600 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "coop_kernel" -d $OUT/pmc_grp_r2r -o p --output-format csv -- python3 $R/scripts/sweep.py --k 4 --backends coop-grp --steps 3 > $OUT/pmc_grp_r2r.jsonl 2> $OUT/pmc_grp_r2r.log || { tail -20 $OUT/pmc_grp_r2r.log; exit 34; }
python3 - <<PY
import csv, glob, collections
f = glob.glob("$OUT/pmc_grp_r2r/**/*counter_collection.csv", recursive=True)[0]
d = collections.defaultdict(dict)
for r in csv.DictReader(open(f)):
    if int(r["Grid_Size"]) >= 10000000:
        d[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
        d[int(r["Dispatch_Id"])]["ms"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        d[int(r["Dispatch_Id"])]["grid"] = int(r["Grid_Size"])
for i, k in enumerate(sorted(d)):
    x = d[k]
    print(i, x["grid"], round(x["ms"], 3), int(x["TCC_EA0_RDREQ_sum"]) / 1e7, int(x["TCC_HIT_sum"]) / 1e7, int(x["TCC_MISS_sum"]) / 1e7)
PY
