#!/bin/bash
# Round-2 session V: smoke() (now with K=4 + remainder), then an N=2 rehearsal
# of the bench on the one-GPU box at 1 Gbase (both ranks share the card, so the
# per-rank K=4 leg must fit twice).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
true
true
cd /tmp
timeout -k 10 700 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 $R/bench.py --gpus 2 --steps 10 --warmup 5 --ref-size 1000000000 --queries 2000000 --config5-queries 2000000 > $OUT/bench_r2v_n2.json 2> $OUT/bench_r2v_n2.log || { tail -30 $OUT/bench_r2v_n2.log; exit 33; }
cut -c1-400 $OUT/bench_r2v_n2.json
python3 - <<PY
import json
b = json.loads(open("$OUT/bench_r2v_n2.json").read().strip().splitlines()[-1])
print(json.dumps(b["variants"].get("kstep4"))[:1500])
PY
cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_kstep4.py tests/test_device_resident.py tests/test_remainder.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r2v.log 2>&1 || { tail -40 $OUT/gpu_tests_r2v.log; exit 34; }
tail -2 $OUT/gpu_tests_r2v.log
cd /tmp
timeout -k 10 300 python3 -u $R/scripts/k4_upload_probe.py > $OUT/k4_upload_r2v.txt 2>&1 || { tail -20 $OUT/k4_upload_r2v.txt; exit 35; }
cat $OUT/k4_upload_r2v.txt
