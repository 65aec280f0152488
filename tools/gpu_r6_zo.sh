#!/bin/bash
# GPU box (round 6): the 1x1 LDS-DMA BN+ReLU-in forward with z_out (ResNet-50 bottleneck conv3) --
# parity, the R50 step vs the oracle with it on, and the config-5 A/B
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6zo
mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_bnrelu_in_glds.py \
  > $o/t1.log 2>&1 || { echo tests failed; tail -30 $o/t1.log; exit 1; }
tail -1 $o/t1.log
SSIP_BNRELU_GLDS=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_semi_step.py -k r50 > $o/t2.log 2>&1 || { echo r50 step failed; tail -30 $o/t2.log; exit 1; }
tail -1 $o/t2.log
bash tools/ab_multi.sh r6zo 3 "SSIP_BNRELU_GLDS=0" "SSIP_BNRELU_GLDS=1" -- --arch resnet50 --image-size 512 --batch 128 --steps 20 || exit 1
