#!/bin/bash
# GPU box (round 6): big budget wgrads -- per-launch at 160 workgroups, then step arms.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6j
mkdir -p $o
timeout -k 10 300 python -u tools/wgrad_lab.py --cfg "default;128,256,2,4,2;256,256,4,2,2" --budgets 160,256 \
  > $o/wgrad_lab.log 2>&1 || { tail -20 $o/wgrad_lab.log; exit 1; }
grep -v amdgpu.ids $o/wgrad_lab.log
bash tools/ab_multi.sh r6j 4 "SSIP_WGRAD_BIG=0" "SSIP_WGRAD_BIG=3 SSIP_WGRAD_BIG_CUS=62" \
  "SSIP_WGRAD_BIG=4 SSIP_WGRAD_BIG_CUS=62" "SSIP_WGRAD_BIG=4 SSIP_WGRAD_BIG_CUS=50"
