#!/bin/bash
# GPU box (round 5): stem pool k3s2 kernel over column groups (any width): parity, config-5 A/B
# (R50 512^2: 128 pooled columns) and the config-5 line with its CPU baseline on the final code.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5ad
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_stem_pool.py tests/test_gpu_c5.py tests/test_gpu_r50_geometry.py > $o/tests.log 2>&1 || { echo tests failed; tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
bash tools/ab_env.sh c5pool "SSIP_POOL_ROWS=0" "SSIP_POOL_ROWS=4" 2 --arch resnet50 --image-size 512 --batch 128 --steps 10 || exit 1
timeout -k 10 900 python bench.py --arch resnet50 --image-size 512 --batch 128 > $o/c5.log 2>&1 || { tail -20 $o/c5.log; exit 1; }
tail -1 $o/c5.log | cut -c1-300
