#!/bin/bash
# GPU box (round 6): CU share of the 8-wave 256x256 budget wgrads (SSIP_WGRAD_BIG=3).
set -o pipefail
export TMPDIR=/tmp
bash tools/ab_multi.sh r6i 4 "SSIP_WGRAD_BIG=0" "SSIP_WGRAD_BIG=3 SSIP_WGRAD_BIG_CUS=25" \
  "SSIP_WGRAD_BIG=3 SSIP_WGRAD_BIG_CUS=37" "SSIP_WGRAD_BIG=3 SSIP_WGRAD_BIG_CUS=50" \
  "SSIP_WGRAD_BIG=3 SSIP_WGRAD_BIG_CUS=62" "SSIP_WGRAD_BIG=3 SSIP_WGRAD_BIG_CUS=75"
