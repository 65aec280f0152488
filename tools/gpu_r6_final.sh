#!/bin/bash
# GPU box (round 6, final tree): the whole -m gpu suite + smoke, then the default bench line
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_r6_full.sh r6final || exit 1
timeout -k 10 500 python bench.py > gpurun_out/r6final/bench.log 2>&1 || { tail -20 gpurun_out/r6final/bench.log; exit 1; }
tail -1 gpurun_out/r6final/bench.log | cut -c1-300
