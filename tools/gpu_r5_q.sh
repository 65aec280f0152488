#!/bin/bash
# GPU box (round 5): one-wave finalize workgroups, more runs.
set -o pipefail
export TMPDIR=/tmp
bash tools/ab_env.sh fin64d "SSIP_FIN64=0" "SSIP_FIN64=1" 5 || exit 1
