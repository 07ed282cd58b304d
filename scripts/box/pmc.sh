#!/bin/bash
# Per-backend fabric read requests (TCC_EA0_RDREQ, TCC_REQ) of the LF kernels, one rocprofv3 --pmc
# pass each: the bench's 10M x 100 bp batch and config #5's 10M x 150 bp shard (seed 20).
#   bash scripts/box/pmc.sh <tag> [q100|q150|both|fetch]
set -o pipefail
T=${1:?tag}
W=${2:-both}
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
run() {  # name, extra args
  local N=$1; shift
  timeout -s KILL 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_REQ_sum --kernel-include-regex "task_kernel|coop_kernel" -d $OUT/pmc_${T}_$N -o p --output-format csv -- python3 $R/scripts/pmc_variants.py --order $OUT/pmc_${T}_${N}_order.json "$@" > $OUT/pmc_${T}_$N.log 2>&1 || { tail -20 $OUT/pmc_${T}_$N.log; return 33; }
  local CSV=$(find $OUT/pmc_${T}_$N -name "*counter_collection.csv" | head -1)
  cp $CSV $OUT/pmc_${T}_${N}.csv
  python3 $R/scripts/traffic_variants.py $CSV $OUT/pmc_${T}_${N}_order.json --source "profiles/${PROF_DIR:-r06}/pmc_${T}_${N}.csv (rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_REQ_sum over scripts/pmc_variants.py $*)" > $OUT/traffic_variants_${T}_$N.json || return 34
  grep -o '"line_requests_per_query": [0-9.]*' $OUT/traffic_variants_${T}_$N.json | head -20
}
if [ "$W" = fetch ]; then
  # the headline kernel's HBM-side bytes by the guide's recipe: FETCH_SIZE in a pass of its own, then
  # the request-size counters (every request 128 B -> FETCH_SIZE x 2), task-mid only
  SIZES="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
  for P in fetch sizes; do
    C=FETCH_SIZE; [ $P = sizes ] && C=$SIZES
    timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex "task_kernel" -d $OUT/pmc_${T}_lf_$P -o p --output-format csv -- python3 $R/scripts/pmc_variants.py --order $OUT/pmc_${T}_lf_${P}_order.json --backends task-mid --k4-backends= > $OUT/pmc_${T}_lf_$P.log 2>&1 || { tail -20 $OUT/pmc_${T}_lf_$P.log; exit 35; }
    CSV=$(find $OUT/pmc_${T}_lf_$P -name "*counter_collection.csv" | head -1)
    cp $CSV $OUT/pmc_${T}_lf_$P.csv || exit 36
    python3 $R/scripts/pmc_summary.py $OUT/pmc_${T}_lf_$P.csv --skip-first > $OUT/pmc_${T}_lf_$P.jsonl || exit 37
    cat $OUT/pmc_${T}_lf_$P.jsonl
  done
  exit 0
fi
if [ "$W" = q100 ] || [ "$W" = both ]; then run q100 || exit $?; fi
if [ "$W" = q150 ] || [ "$W" = both ]; then
  run q150 --qlen 150 --seed 20 --backends task-mid,coop-mid,task,coop,task-ac,task-ac-mid --k4-backends coop-grp || exit $?
fi
