#!/bin/bash
# GPU box (round 5): stem conv ablations (SSIP_STEM_DIAG: 1 no stores, 2 no wait after the k-loop,
# 8 no BN statistics, combinations).
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/halo_lab.py --stem-diags 0,2,1,3,8,11 --batches 256 2>&1 | grep -v amdgpu.ids | grep stem
