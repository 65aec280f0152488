#!/bin/bash
# GPU box (round 6): re-check the step's older scheduling knobs under the round-6 defaults.
set -o pipefail
export TMPDIR=/tmp
bash tools/ab_multi.sh r6p 3 "SSIP_X=0" "SSIP_FUSE_BN_BWD=halo" "SSIP_FUSE_BN_BWD=0" "SSIP_FIN64=1" \
  "SSIP_MAX_INFLIGHT=3" "SSIP_LAST_WG_FULL=1" || exit 1
