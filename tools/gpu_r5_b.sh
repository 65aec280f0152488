#!/bin/bash
# GPU box (round 5): fused stem conv + pool -- parity, lab, step A/B.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5b
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_stem_pool.py tests/test_gpu_semi_step.py tests/test_gpu_bench_geometry.py tests/test_gpu_halo.py \
  > $o/tests.log 2>&1 || { echo tests failed; tail -40 $o/tests.log; exit 1; }
tail -2 $o/tests.log
bash tools/ab_env.sh stempool "SSIP_STEM_POOL=1" "SSIP_STEM_POOL=0" 3 || exit 1
bash tools/ab_env.sh wgbig2 "SSIP_WGRAD_BIG=2" "SSIP_WGRAD_BIG=0" 2 || exit 1
