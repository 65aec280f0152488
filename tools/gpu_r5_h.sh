#!/bin/bash
# GPU box (round 5): halo fwd/dgrad with the next tile's DMA pieces among the MFMAs
# (SSIP_HALO_DIAG=16: ahead of them, as before): parity, lab, step A/B.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5h
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_halo.py tests/test_gpu_conv.py tests/test_gpu_eval_fold.py tests/test_gpu_block_fusion.py \
  tests/test_gpu_resnet.py > $o/tests.log 2>&1 || { echo tests failed; tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
timeout -k 10 300 python -u tools/halo_lab.py --diags 0,16,4,8 > $o/halo.log 2>&1 || { echo halo lab failed; tail -5 $o/halo.log; exit 1; }
grep -v amdgpu.ids $o/halo.log
bash tools/ab_env.sh spread "SSIP_HALO_DIAG=16" "SSIP_HALO_DIAG=0" 3 || exit 1
