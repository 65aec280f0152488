#!/bin/bash
# GPU box (round 6): the new default budget wgrads -- bench-geometry wgrad parity, step bit-identity /
# plan tests, DP tests; config-5 A/B of the mode.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6l
mkdir -p $o
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_bench_geometry.py tests/test_gpu_semi_step.py tests/test_gpu_dist.py tests/test_gpu_rccl.py \
  -k "wgrad or plan or graph or bit_identical or dp2 or rccl or early" > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
grep -E "PASS|FAIL" $o/tests.log | tail -50
bash tools/ab_env.sh r6l_c5 "SSIP_WGRAD_BIG=0" "SSIP_WGRAD_BIG=4" 2 --arch resnet50 --image-size 512 --batch 128 || exit 1
