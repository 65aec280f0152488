#!/bin/bash
# GPU box (round 6): HIP runtime knobs for the plan-replayed step (kernel arguments in device memory)
set -o pipefail
export TMPDIR=/tmp
bash tools/ab_multi.sh r6z 3 "SSIP_NONE=1" "HIP_FORCE_DEV_KERNARG=1" "HIP_FORCE_DEV_KERNARG=0" || exit 1
