#!/bin/bash
# GPU box (round 5): stem pool forward, ymax from LDS slots vs per-tap selects, step A/B.
set -o pipefail
export TMPDIR=/tmp
bash tools/ab_env.sh poollds "SSIP_POOL_LDS=0" "SSIP_POOL_LDS=1" 3 || exit 1
