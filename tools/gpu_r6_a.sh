#!/bin/bash
# GPU box (round 6): the conv_glds stagger -- per-launch lab (bitwise + alternated timing), the new
# parity tests (ABI-13 kernels at the bench geometry, real-data N1, step bit-identity), then a step A/B.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6a
timeout -k 10 400 python -u tools/stagger_lab.py --rounds 3 > gpurun_out/r6a/lab.log 2>&1 || { tail -20 gpurun_out/r6a/lab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6a/lab.log
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_real_data.py tests/test_gpu_bench_geometry.py -k "bnrelu or k3s2 or real" \
  > gpurun_out/r6a/tests1.log 2>&1 || { tail -40 gpurun_out/r6a/tests1.log; exit 1; }
grep -E "PASS|FAIL|max \|P" gpurun_out/r6a/tests1.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_semi_step.py -k "bit_identical" > gpurun_out/r6a/tests2.log 2>&1 || { tail -40 gpurun_out/r6a/tests2.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/r6a/tests2.log
bash tools/ab_env.sh r6a_step "SSIP_STAGGER=0" "SSIP_STAGGER=7" 3
