#!/bin/bash
# GPU box (round 5): mid-step ring refill for the 256x256 tiles only (SSIP_DMA_MID=2).
set -o pipefail
export TMPDIR=/tmp
bash tools/ab_env.sh dmamid2 "SSIP_DMA_MID=0" "SSIP_DMA_MID=2" 4 || exit 1
