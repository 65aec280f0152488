#!/bin/bash
# GPU box (round 5): where the BN+ReLU-in forward's extra time goes (SSIP_HALO_DIAG ablations).
set -o pipefail
export TMPDIR=/tmp
for d in 0 32 64 96 4; do
  echo "-- diag $d"; SSIP_HALO_DIAG=$d timeout -k 10 120 python -u tools/bnrelu_in_lab.py 2>&1 | grep -v amdgpu.ids | grep "fwd"
done
