#!/bin/bash
# GPU box (round 5): halo dgrad epilogue operands (residual / BN-backward y) requested at tile
# start vs after the MFMAs (tools/lab/base build): parity, lab for both, step A/B.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5i
mkdir -p $o
B=$PWD/tools/lab/base/libssip_hip.so
N=$PWD/semi-supervised-image-processing_amd/ssip/libssip_hip.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_halo.py tests/test_gpu_conv.py tests/test_gpu_eval_fold.py tests/test_gpu_block_fusion.py \
  tests/test_gpu_resnet.py tests/test_gpu_semi_step.py > $o/tests.log 2>&1 || { echo tests failed; tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
for v in new base; do
  if [ $v = base ]; then L=$B; else L=$N; fi
  SSIP_LIB=$L timeout -k 10 300 python -u tools/halo_lab.py --diags 0 > $o/halo_$v.log 2>&1 || { echo halo lab failed; tail -5 $o/halo_$v.log; exit 1; }
  echo "== $v"; grep -v "amdgpu.ids\|stem\|pooled" $o/halo_$v.log
done
bash tools/ab_env.sh prefetch "SSIP_LIB=$B" "SSIP_LIB=$N" 3 || exit 1
