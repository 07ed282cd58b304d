#!/bin/bash
# Round-1 session ZK: profile refresh on the final build -- default bench
# (warmup 20), rocprofv3 kernel stats of the headline run, one TCC PMC pass.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 700 python3 $R/bench.py > $OUT/bench_r01zk.json 2> $OUT/bench_r01zk.log || { tail -20 $OUT/bench_r01zk.log; exit 31; }
python3 -c "import json; d=json.load(open('$OUT/bench_r01zk.json')); v=d['variants']; print(d['value'], d['ms_per_step'], d['roofline']['lf_ms'], d['roofline']['frac'], d['cpu_baseline']['value'], {k: (x.get('mqps') if isinstance(x, dict) else x) for k, x in v.items()})"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_r01zk -o bench --output-format csv -- python3 $R/bench.py --no-config1 --variants "" --cpu-sample 0 --e2e-steps 0 --sa-rate 0 > $OUT/prof_bench_r01zk.json 2> $OUT/prof_bench_r01zk.log || exit 33
echo prof_done
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_DRAM_sum --kernel-include-regex "task_kernel" -d $OUT/pmc_r01zk -o p --output-format csv -- python3 $R/scripts/sweep.py --backends task-mid --steps 2 > $OUT/pmc_r01zk.jsonl 2> $OUT/pmc_r01zk.log || exit 34
echo pmc_done
