#!/bin/bash
# GPU box (round 5): stem pool forward k3s2: ymax from LDS slots, rows per workgroup.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5v
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_stem_pool.py > $o/tests.log 2>&1 || { echo tests failed; tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
timeout -k 10 120 python -u tools/pool_lab.py --rows 4,8,16 --lds 0,1 > $o/lab.log 2>&1 || { tail -5 $o/lab.log; exit 1; }
grep -v amdgpu.ids $o/lab.log
