#!/bin/bash
# GPU box (round 6): HIP / HSA runtime knobs for the plan-replayed step
set -o pipefail
export TMPDIR=/tmp
bash tools/ab_multi.sh r6z2 3 "SSIP_NONE=1" "GPU_MAX_HW_QUEUES=8" "HSA_ENABLE_INTERRUPT=0" "AMD_DIRECT_DISPATCH=0" || exit 1
