#!/bin/bash
# GPU box (round 6): config 5 (ResNet-50 512^2 bs128) knob re-check under the round-6 defaults
set -o pipefail
export TMPDIR=/tmp
bash tools/ab_multi.sh r6x 3 "SSIP_NONE=1" "SSIP_WGRAD_BIG_CUS=50" "SSIP_WGRAD_BIG_CUS=75" "SSIP_STAGGER=0" \
  "SSIP_BNRELU_GLDS=1" "SSIP_WGRAD_BIG=3" -- --arch resnet50 --image-size 512 --batch 128 --steps 20
