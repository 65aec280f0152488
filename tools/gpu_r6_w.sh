#!/bin/bash
# GPU box (round 6): 4-wave (2x2) 128x128 LDS-DMA tiles vs the planner's, per launch (bits compared), fwd/dgrad/wgrad
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6w
mkdir -p $o
timeout -k 10 400 python -u tools/tile_force_lab.py --cfg "128,128,2,2,2" --modes fd \
  --shapes l2.3x3s2,l2.3x3,l2.ds,l3.3x3s2,l3.3x3,l3.ds,l4.3x3s2,l4.3x3,l4.ds > $o/fd.log 2>&1 || { tail -20 $o/fd.log; exit 1; }
grep -v amdgpu.ids $o/fd.log
timeout -k 10 400 python -u tools/wgrad_lab.py --cfg "default;128,128,2,2,2" --budgets 0,256 > $o/wg.log 2>&1 || { tail -20 $o/wg.log; exit 1; }
grep -v amdgpu.ids $o/wg.log
