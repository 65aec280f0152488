#!/bin/bash
# GPU box (round 5): step-boundary copy engine (HSA_ENABLE_SDMA=0: the H2D view-parameter copy as a
# blit kernel) A/B.
set -o pipefail
export TMPDIR=/tmp
bash tools/ab_env.sh sdma "HSA_ENABLE_SDMA=1" "HSA_ENABLE_SDMA=0" 3 || exit 1
