#!/bin/bash
# GPU box: the main-loop lab, then a short bench line.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-lab}
mkdir -p $o
timeout -k 10 120 ./tools/lab/gemm_lab 20 > $o/lab.log 2>&1 || { echo lab failed; tail -5 $o/lab.log; exit 1; }
cat $o/lab.log
timeout -k 10 420 python bench.py --cpu-warmup 1 --cpu-steps 3 > $o/bench.log 2>&1 || { echo bench failed; tail -5 $o/bench.log; exit 1; }
tail -1 $o/bench.log
