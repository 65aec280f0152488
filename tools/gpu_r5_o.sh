#!/bin/bash
# GPU box (round 5): stem conv store / statistics ablations.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5o
mkdir -p $o
timeout -k 10 300 python -u tools/halo_lab.py --diags 0 --stem-diags 0,1,8,9 --batches 256 > $o/halo.log 2>&1 || { tail -5 $o/halo.log; exit 1; }
grep -v amdgpu.ids $o/halo.log
