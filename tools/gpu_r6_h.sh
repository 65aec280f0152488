#!/bin/bash
# GPU box (round 6): step A/B of the 8-wave 256x256 budget wgrads (SSIP_WGRAD_BIG=3) on all / half the CUs.
set -o pipefail
export TMPDIR=/tmp
bash tools/ab_env.sh r6h_big "SSIP_WGRAD_BIG=0" "SSIP_WGRAD_BIG=3" 3 || exit 1
bash tools/ab_env.sh r6h_big50 "SSIP_WGRAD_BIG=0" "SSIP_WGRAD_BIG=3 SSIP_WGRAD_BIG_CUS=50" 3 || exit 1
