#!/bin/bash
# GPU box (round 6): what the BN finalize launches cost the step (timing-only skips, results wrong)
set -o pipefail
export TMPDIR=/tmp
bash tools/ab_multi.sh r6fin 3 "SSIP_NONE=1" "SSIP_DIAG_NO_BWD_FIN=1" "SSIP_DIAG_NO_FWD_FIN=1" \
  "SSIP_DIAG_NO_BWD_FIN=1 SSIP_DIAG_NO_FWD_FIN=1" || exit 1
