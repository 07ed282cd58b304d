#!/bin/bash
# Round-3 session P: coop on the reference layouts with the counter words
# loaded after the DMA in two 32-lane groups -- parity, then the sweep.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_alphabet.py tests/test_gpu_fullscale.py -m gpu -x -q -k "coop or index_md5" --timeout 600 --timeout-method thread -p no:cacheprovider > $OUT/p_parity.log 2>&1 || { tail -40 $OUT/p_parity.log; exit 31; }
tail -2 $OUT/p_parity.log
cd /tmp
timeout -k 10 600 python3 -u $R/scripts/sweep.py --backends coop,coop-ac,coop-mid --steps 10 > $OUT/sweep_r3p.jsonl 2> $OUT/sweep_r3p.log || { tail -30 $OUT/sweep_r3p.log; exit 33; }
cut -c1-170 $OUT/sweep_r3p.jsonl
