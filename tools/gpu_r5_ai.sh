#!/bin/bash
# GPU box (round 5, final code): BN-backward fusion policy re-check (default vs every halo dgrad).
set -o pipefail
export TMPDIR=/tmp
bash tools/ab_env.sh fusehalo "SSIP_FUSE_BN_BWD=" "SSIP_FUSE_BN_BWD=halo" 4 || exit 1
