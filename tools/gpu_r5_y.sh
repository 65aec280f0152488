#!/bin/bash
# GPU box (round 5, after the BN+ReLU-in and pool changes): one-wave finalize, halo wgrad CU share.
set -o pipefail
export TMPDIR=/tmp
bash tools/ab_env.sh fin64e "SSIP_FIN64=0" "SSIP_FIN64=1" 4 || exit 1
bash tools/ab_env.sh hwg375 "SSIP_HALO_WG_FRAC=0.5" "SSIP_HALO_WG_FRAC=0.375" 3 || exit 1
bash tools/ab_env.sh hwg625 "SSIP_HALO_WG_FRAC=0.5" "SSIP_HALO_WG_FRAC=0.625" 3 || exit 1
