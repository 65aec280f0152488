#!/bin/bash
# GPU box: sweep of the side-stream halo wgrad grid (percent of the CU budget)
set -o pipefail
bash tools/ab_multi.sh halopct 3 "SSIP_HALO_WG_PCT=100" "SSIP_HALO_WG_PCT=25" "SSIP_HALO_WG_PCT=37" "SSIP_HALO_WG_PCT=50" "SSIP_HALO_WG_PCT=62"
