#!/bin/bash
# GPU box (round 5): halo wgrad with the next tile's DMA pieces among the MFMAs
# (SSIP_HWG_SPREAD=0: ahead of them): parity, per-launch times, step A/B.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5j
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_halo.py tests/test_gpu_conv.py tests/test_gpu_resnet.py tests/test_gpu_semi_step.py \
  tests/test_gpu_bench_geometry.py > $o/tests.log 2>&1 || { echo tests failed; tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
for v in 1 0; do
  SSIP_HWG_SPREAD=$v timeout -k 10 300 python -u tools/conv_times.py --modes w > $o/wg_$v.log 2>&1 || { echo conv_times failed; tail -5 $o/wg_$v.log; exit 1; }
  echo "== spread $v"; grep "l1.3x3" $o/wg_$v.log
done
bash tools/ab_env.sh hwgspread "SSIP_HWG_SPREAD=0" "SSIP_HWG_SPREAD=1" 3 || exit 1
