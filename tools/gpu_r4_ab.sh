#!/bin/bash
# GPU box: per-launch conv breakdown of the in-tree library against ab/libssip_base.so
# (alternated), then the main-loop lab.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-ablaunch}
mkdir -p $o
for i in 1 2; do
  SSIP_LIB=ab/libssip_base.so timeout -k 10 300 python tools/conv_breakdown.py > $o/base$i.log 2>&1 || { echo base failed; tail -5 $o/base$i.log; exit 1; }
  timeout -k 10 300 python tools/conv_breakdown.py > $o/new$i.log 2>&1 || { echo new failed; tail -5 $o/new$i.log; exit 1; }
  echo "run $i base: $(tail -1 $o/base$i.log)"; echo "run $i new:  $(tail -1 $o/new$i.log)"
done
timeout -k 10 120 ./tools/lab/gemm_lab 20 > $o/lab.log 2>&1 || { echo lab failed; tail -5 $o/lab.log; exit 1; }
cat $o/lab.log
