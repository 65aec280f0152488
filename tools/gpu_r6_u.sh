#!/bin/bash
# GPU box (round 6): halo forward phase stamps under ablations
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6u
timeout -k 10 180 python -u tools/halo_stamp_lab.py --diags 0,1,2,3,8,11,15 --out gpurun_out/r6u/stamps.txt > gpurun_out/r6u/stamps.log 2>&1 || { tail -20 gpurun_out/r6u/stamps.log; exit 1; }
cat gpurun_out/r6u/stamps.txt
