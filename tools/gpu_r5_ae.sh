#!/bin/bash
# GPU box (round 5): layer-1 halo wgrad CU share 0.5 vs 0.625, 5 + 5 runs.
set -o pipefail
export TMPDIR=/tmp
bash tools/ab_env.sh hwg625b "SSIP_HALO_WG_FRAC=0.5" "SSIP_HALO_WG_FRAC=0.625" 5 || exit 1
