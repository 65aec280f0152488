#!/bin/bash
# GPU box: launch-plan replays in flight (host bound), re-checked at the end of round 4
set -o pipefail
bash tools/ab_multi.sh inflight 3 "SSIP_MAX_INFLIGHT=2" "SSIP_MAX_INFLIGHT=3" "SSIP_MAX_INFLIGHT=4"
