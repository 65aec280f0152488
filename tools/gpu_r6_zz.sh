#!/bin/bash
# GPU box (round 6): R18 re-checks under the final defaults -- halo z_out (SSIP_BNRELU_Z), stagger masks
set -o pipefail
export TMPDIR=/tmp
bash tools/ab_multi.sh r6zz 3 "SSIP_NONE=1" "SSIP_BNRELU_Z=1" "SSIP_STAGGER=6" "SSIP_STAGGER=3" || exit 1
