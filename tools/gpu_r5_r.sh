#!/bin/bash
# GPU box (round 5): layer-1 BN+ReLU applied inside the next conv (ABI 13): parity, step A/B.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5r
mkdir -p $o
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_bnrelu_in.py tests/test_gpu_halo.py tests/test_gpu_semi_step.py tests/test_gpu_resnet.py \
  tests/test_gpu_bench_geometry.py tests/test_gpu_block_fusion.py tests/test_gpu_r50_geometry.py > $o/tests.log 2>&1 || { echo tests failed; tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
bash tools/ab_env.sh bnrin "SSIP_BNRELU_IN=0" "SSIP_BNRELU_IN=1" 4 || exit 1
