#!/bin/bash
# GPU box: A/B of the wgrad grid size (SSIP_WGRAD_BLOCKS: target workgroups per wgrad launch)
set -o pipefail
export TMPDIR=/tmp
bash tools/ab_env.sh wgb256 "SSIP_AB_BASE=1" "SSIP_WGRAD_BLOCKS=256" 3 || exit 1
