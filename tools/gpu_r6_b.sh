#!/bin/bash
# GPU box (round 6): stagger step A/B, then the new parity tests with diagnostics.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6b
bash tools/ab_env.sh r6b_step "SSIP_STAGGER=0" "SSIP_STAGGER=7" 3 || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_semi_step.py -k "bit_identical" > gpurun_out/r6b/tests2.log 2>&1 || { tail -40 gpurun_out/r6b/tests2.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/r6b/tests2.log
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_real_data.py tests/test_gpu_bench_geometry.py -k "bnrelu or k3s2 or real" \
  > gpurun_out/r6b/tests1.log 2>&1; rc=$?
grep -E "PASS|FAIL|max dP|flips|_loss|Error" gpurun_out/r6b/tests1.log | head -60
exit $rc
