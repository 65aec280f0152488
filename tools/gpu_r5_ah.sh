#!/bin/bash
# GPU box (round 5): stem conv stores through LDS (16-B) vs 2-byte stores (SSIP_STEM_DIAG=4): parity,
# lab, step A/B.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5ah
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_conv.py tests/test_gpu_bench_geometry.py tests/test_gpu_halo.py tests/test_gpu_semi_step.py tests/test_gpu_c5.py > $o/tests.log 2>&1 || { echo tests failed; tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
timeout -k 10 200 python -u tools/halo_lab.py --stem-diags 0,4,1 --batches 256,128 2>&1 | grep -v amdgpu.ids | grep stem
bash tools/ab_env.sh stemst "SSIP_STEM_DIAG=4" "SSIP_STEM_DIAG=0" 4 || exit 1
