#!/bin/bash
# GPU box (round 5): halo TX epilogue + budget wgrad tiles -- parity first, then labs and a step A/B.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5a
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_halo.py tests/test_gpu_bench_geometry.py tests/test_gpu_eval_fold.py tests/test_gpu_block_fusion.py \
  > $o/tests.log 2>&1 || { echo tests failed; tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
timeout -k 10 300 python -u tools/halo_lab.py > $o/halo.log 2>&1 || { echo halo lab failed; tail -5 $o/halo.log; exit 1; }
cat $o/halo.log
bash tools/ab_env.sh halotx "SSIP_HALO_TX=1" "SSIP_HALO_TX=0" 2 || exit 1
bash tools/ab_env.sh wgbig "SSIP_WGRAD_BIG=1" "SSIP_WGRAD_BIG=0" 2 || exit 1
