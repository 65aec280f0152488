#!/bin/bash
# GPU box: the main-loop lab (tools/lab/gemm_lab, built on the CPU host), then a short bench line.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/lab
mkdir -p $o
timeout -k 10 120 ./tools/lab/gemm_lab ${1:-20} > $o/lab.log 2>&1; rc=$?
cat $o/lab.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --cpu-warmup 1 --cpu-steps 3 > $o/bench.log 2>&1 || { echo bench failed; tail -5 $o/bench.log; exit 1; }
tail -1 $o/bench.log
