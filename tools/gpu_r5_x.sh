#!/bin/bash
# GPU box (round 5): augment ToTensor/jitter/Normalize tables: parity, step A/B against a library
# built with the previous augment kernel (abtmp/libssip_old.so, built on the CPU side).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5x
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_augment.py tests/test_gpu_semi_step.py tests/test_gpu_pipeline.py > $o/tests.log 2>&1 || { echo tests failed; tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
bash tools/ab_env.sh auglut "SSIP_LIB=$PWD/abtmp/libssip_old.so" "SSIP_AUG_NEW=1" 3 || exit 1
