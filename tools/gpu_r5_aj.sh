#!/bin/bash
# GPU box (round 5): BN+ReLU-in forward writing z for a plain layer-1 wgrad (SSIP_BNRELU_Z): parity,
# lab, step A/B.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5aj
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_bnrelu_in.py tests/test_gpu_halo.py tests/test_gpu_semi_step.py tests/test_gpu_resnet.py tests/test_gpu_bench_geometry.py > $o/tests.log 2>&1 || { echo tests failed; tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
bash tools/ab_env.sh bnrz "SSIP_BNRELU_Z=0" "SSIP_BNRELU_Z=1" 4 || exit 1
