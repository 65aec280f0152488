#!/bin/bash
# GPU box (round 5): budget wgrads on 8-wave 128x256 tiles (SSIP_WGRAD_BIG=3): parity, lab, step A/B.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5p
mkdir -p $o
SSIP_WGRAD_BIG=3 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_bench_geometry.py tests/test_gpu_semi_step.py tests/test_gpu_conv.py > $o/tests.log 2>&1 || { echo tests failed; tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
timeout -k 10 300 python -u tools/wgrad_lab.py --cfg "default;128,256,2,4,2" --budgets 256 > $o/wlab.log 2>&1 || { tail -5 $o/wlab.log; exit 1; }
grep -v amdgpu.ids $o/wlab.log
bash tools/ab_env.sh wgbig3 "SSIP_WGRAD_BIG=0" "SSIP_WGRAD_BIG=3" 4 || exit 1
