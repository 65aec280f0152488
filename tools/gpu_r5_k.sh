#!/bin/bash
# GPU box (round 5): layer-1 wgrad CU share after the wgrad DMA change.
set -o pipefail
export TMPDIR=/tmp
bash tools/ab_env.sh hwgfrac75 "SSIP_HALO_WG_FRAC=0.5" "SSIP_HALO_WG_FRAC=0.75" 3 || exit 1
bash tools/ab_env.sh hwgfrac100 "SSIP_HALO_WG_FRAC=0.5" "SSIP_HALO_WG_FRAC=1.0" 2 || exit 1
