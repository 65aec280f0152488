#!/bin/bash
# GPU box: re-sweep of the side-stream wgrad workgroup target after the coalesced slab reduce
set -o pipefail
bash tools/ab_multi.sh wgb3 3 "SSIP_X=0" "SSIP_WGRAD_BLOCKS=192" "SSIP_WGRAD_BLOCKS=384" "SSIP_WGRAD_BLOCKS=512"
