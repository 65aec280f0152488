#!/bin/bash
# GPU box (round 6): the 1x1 BN+ReLU-in row threshold -- its tests, the R50 step vs the oracle, config-5 A/B
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6mm
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bnrelu_in_glds.py \
  tests/test_gpu_c5.py tests/test_gpu_r50_geometry.py tests/test_gpu_semi_step.py > $o/t.log 2>&1 || { echo tests failed; tail -30 $o/t.log; exit 1; }
tail -1 $o/t.log
bash tools/ab_multi.sh r6mm 3 "SSIP_NONE=1" "SSIP_BNRELU_GLDS_MINM=0" -- --arch resnet50 --image-size 512 --batch 128 --steps 20 || exit 1
