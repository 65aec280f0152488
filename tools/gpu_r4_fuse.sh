#!/bin/bash
# GPU box: BN-backward fusion policy re-checked after round 4's co-scheduling changes
set -o pipefail
bash tools/ab_multi.sh fuse4 3 "SSIP_X=0" "SSIP_FUSE_BN_BWD=halo" "SSIP_FUSE_BN_BWD=0" "SSIP_FUSE_BN_BWD=1"
