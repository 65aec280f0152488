#!/bin/bash
# GPU box (round 6): re-sweep the side stream's CU shares and older scheduling knobs under the round-6
# defaults (one box, alternated); config-5 A/B of the wide budget wgrads.
set -o pipefail
export TMPDIR=/tmp
bash tools/ab_multi.sh r6o 3 "SSIP_X=0" "SSIP_HALO_WG_FRAC=0.375" "SSIP_HALO_WG_FRAC=0.625" \
  "SSIP_WGRAD_BIG_CUS=56" "SSIP_WGRAD_BIG_CUS=66" "SSIP_FUSE_BN_BWD=halo" "SSIP_FUSE_BN_BWD=0" "SSIP_FIN64=1" \
  "SSIP_MAX_INFLIGHT=3" "SSIP_LAST_WG_FULL=1" "SSIP_DMA_MID=1" "SSIP_DMA_MID=2" || exit 1
bash tools/ab_env.sh r6o_c5 "SSIP_WGRAD_BIG=0" "SSIP_WGRAD_BIG=4" 2 --arch resnet50 --image-size 512 --batch 128 || exit 1
