#!/bin/bash
# GPU box (round 6, final tree with the 1x1 BN+ReLU-in default): whole -m gpu suite + smoke, the config-5
# line and the default line
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_r6_full.sh r6final2 || exit 1
o=gpurun_out/r6final2
timeout -k 10 400 python bench.py --no-cpu-baseline --arch resnet50 --image-size 512 --batch 128 > $o/c5.log 2>&1 || { tail -20 $o/c5.log; exit 1; }
tail -1 $o/c5.log | cut -c1-200
timeout -k 10 500 python bench.py > $o/bench.log 2>&1 || { tail -20 $o/bench.log; exit 1; }
tail -1 $o/bench.log | cut -c1-200
