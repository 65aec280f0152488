#!/bin/bash
# GPU box (round 5): LDS-DMA ring refill after the k-step's fragment reads (SSIP_DMA_MID=1)
# vs at the step start: parity with it on, per-launch conv times, step A/B.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5m
mkdir -p $o
SSIP_DMA_MID=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_conv.py tests/test_gpu_fwd_ds.py tests/test_gpu_block_fusion.py tests/test_gpu_semi_step.py \
  > $o/tests.log 2>&1 || { echo tests failed; tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
for v in 0 1; do
  SSIP_DMA_MID=$v timeout -k 10 300 python -u tools/conv_times.py > $o/ct_$v.log 2>&1 || { echo conv_times failed; tail -5 $o/ct_$v.log; exit 1; }
done
paste <(awk '{print $1, $2, $3}' $o/ct_0.log) <(awk '{print $3}' $o/ct_1.log) | grep -v amdgpu
bash tools/ab_env.sh dmamid "SSIP_DMA_MID=0" "SSIP_DMA_MID=1" 3 || exit 1
