#!/bin/bash
# GPU box (round 5): the stem pool forward's k3s2 kernel: parity, lab, step A/B.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5u
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_stem_pool.py tests/test_gpu_ops.py tests/test_gpu_c5.py tests/test_gpu_halo.py > $o/tests.log 2>&1 || { echo tests failed; tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
timeout -k 10 120 python -u tools/pool_lab.py > $o/lab.log 2>&1 || { tail -5 $o/lab.log; exit 1; }
grep -v amdgpu.ids $o/lab.log
bash tools/ab_env.sh poolk3 "SSIP_POOL_ROWS=0" "SSIP_POOL_ROWS=4" 3 || exit 1
