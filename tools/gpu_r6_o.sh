#!/bin/bash
# GPU box (round 6): re-sweep the side stream's CU shares with the wide budget wgrads on; config-5 A/B of them.
set -o pipefail
export TMPDIR=/tmp
bash tools/ab_multi.sh r6o 4 "SSIP_X=0" "SSIP_HALO_WG_FRAC=0.375" "SSIP_HALO_WG_FRAC=0.625" \
  "SSIP_WGRAD_BIG_CUS=56" "SSIP_WGRAD_BIG_CUS=66" || exit 1
bash tools/ab_env.sh r6o_c5 "SSIP_WGRAD_BIG=0" "SSIP_WGRAD_BIG=4" 2 --arch resnet50 --image-size 512 --batch 128 || exit 1
