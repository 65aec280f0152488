#!/bin/bash
# GPU box (round 5): config-5 line (R50 512^2, 64 + 64, with its CPU baseline) and the extraction line.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5c5
mkdir -p $o
timeout -k 10 900 python bench.py --arch resnet50 --image-size 512 --batch 128 > $o/c5.log 2>&1 || { tail -20 $o/c5.log; exit 1; }
tail -1 $o/c5.log | cut -c1-300
timeout -k 10 500 python bench.py --workload extract > $o/ex.log 2>&1 || { tail -20 $o/ex.log; exit 1; }
tail -1 $o/ex.log | cut -c1-300
