#!/bin/bash
# GPU box (round 6): halo forward phase stamps
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6s
timeout -k 10 120 python -u tools/halo_stamp_lab.py --out gpurun_out/r6s/stamps.txt > gpurun_out/r6s/stamps.log 2>&1 || { tail -20 gpurun_out/r6s/stamps.log; exit 1; }
cat gpurun_out/r6s/stamps.txt
