#!/bin/bash
# GPU box: single-stream per-launch cost of the one-workgroup-per-CU wgrad grid, and its R50 step A/B
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/wgb2
mkdir -p $o
for i in 1 2; do
  timeout -k 10 300 python tools/conv_breakdown.py > $o/base$i.log 2>&1 || { echo base failed; tail -5 $o/base$i.log; exit 1; }
  SSIP_WGRAD_BLOCKS=256 timeout -k 10 300 python tools/conv_breakdown.py > $o/w256_$i.log 2>&1 || { echo w256 failed; exit 1; }
  echo "run $i base: $(tail -1 $o/base$i.log)"; echo "run $i w256: $(tail -1 $o/w256_$i.log)"
done
bash tools/ab_multi.sh wgb50 2 "SSIP_AB_BASE=1" "SSIP_WGRAD_BLOCKS=256" -- --arch resnet50 --image-size 512 --batch 128 --steps 15 || exit 1
