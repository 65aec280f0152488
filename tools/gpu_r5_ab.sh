#!/bin/bash
# GPU box (round 5): copy-ahead of the view parameters (plan replays): parity, step A/B.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5ab
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_semi_step.py tests/test_gpu_rccl.py tests/test_gpu_pipeline.py > $o/tests.log 2>&1 || { echo tests failed; tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
bash tools/ab_env.sh cpahead "SSIP_COPY_AHEAD=0" "SSIP_COPY_AHEAD=1" 4 || exit 1
