#!/bin/bash
# GPU box (round 6): BN-backward finalize fused into the reduce launch -- its tests, the whole -m gpu
# suite + smoke, and the step A/B against the separate finalize (SSIP_BWD_FIN_FUSE=0)
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6bf
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bn_bwd_fused_fin.py \
  > $o/fused.log 2>&1 || { echo fused tests failed; tail -30 $o/fused.log; exit 1; }
tail -1 $o/fused.log
bash tools/gpu_r6_full.sh r6bf/full || exit 1
bash tools/ab_env.sh r6bf "SSIP_BWD_FIN_FUSE=0" "SSIP_BWD_FIN_FUSE=1" 3 || exit 1
