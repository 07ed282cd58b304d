#!/bin/bash
# round 4a: bench.py --gpus N self-spawn rehearsals on the one-card box (1 Gbase)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
timeout -k 10 400 python3 bench.py --gpus 2 --ref-size 1000000000 --no-kstep4 --steps 10 --warmup 10 \
    > gpurun_out/r4a_n2.json 2> gpurun_out/r4a_n2.log && \
timeout -k 10 600 python3 bench.py --gpus 8 --ref-size 1000000000 --no-kstep4 --steps 10 --warmup 10 \
    > gpurun_out/r4a_n8.json 2> gpurun_out/r4a_n8.log
