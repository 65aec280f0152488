#!/bin/bash
# GPU box (round 6): the config-5 (ResNet-50 512^2 bs128) one-lease profile, then the fp32, extraction
# and default (with CPU baseline) bench lines.
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_r6_prof.sh r6r50 --arch resnet50 --image-size 512 --batch 128 || exit 1
out=gpurun_out/r6lines
mkdir -p $out
timeout -k 10 300 python bench.py --dtype fp32 --no-cpu-baseline > $out/fp32.log 2>&1 || { tail -20 $out/fp32.log; exit 1; }
tail -1 $out/fp32.log | cut -c1-200
timeout -k 10 300 python bench.py --workload extract > $out/extract.log 2>&1 || { tail -20 $out/extract.log; exit 1; }
tail -1 $out/extract.log | cut -c1-200
timeout -k 10 400 python bench.py > $out/default.log 2>&1 || { tail -20 $out/default.log; exit 1; }
tail -1 $out/default.log | cut -c1-200
echo "lines done"
