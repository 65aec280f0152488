#!/bin/bash
# GPU box (round 6): CU share of the mode-4 budget wgrads (8-wave 256x256 for K >= 256, 128x256 for K = 128).
set -o pipefail
export TMPDIR=/tmp
bash tools/ab_multi.sh r6k 4 "SSIP_WGRAD_BIG=0" "SSIP_WGRAD_BIG=4 SSIP_WGRAD_BIG_CUS=56" \
  "SSIP_WGRAD_BIG=4 SSIP_WGRAD_BIG_CUS=62" "SSIP_WGRAD_BIG=4 SSIP_WGRAD_BIG_CUS=70" "SSIP_WGRAD_BIG=4 SSIP_WGRAD_BIG_CUS=80"
