#!/bin/bash
# GPU box (round 5): no argmax bytes in the weak forward's stem pool: parity.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5af
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_stem_pool.py tests/test_gpu_ops.py tests/test_gpu_semi_step.py tests/test_gpu_c5.py > $o/tests.log 2>&1 || { echo tests failed; tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
