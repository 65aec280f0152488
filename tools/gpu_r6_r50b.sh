#!/bin/bash
# GPU box (round 6, final defaults): config-5 one-lease profile again (line, legs, PMC traffic per BN pass)
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_r6_prof.sh r6r50b --arch resnet50 --image-size 512 --batch 128 || exit 1
