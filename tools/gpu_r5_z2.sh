#!/bin/bash
# GPU box (round 5): BN+ReLU-in forward with the transform inside the k-loop (default) vs after it
# (SSIP_HALO_DIAG=32): parity, lab, step A/B.  (Second version: pieces staged through registers.)
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5z4
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_bnrelu_in.py tests/test_gpu_halo.py > $o/tests.log 2>&1 || { echo tests failed; tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
echo "-- after the k-loop"; SSIP_HALO_DIAG=32 timeout -k 10 120 python -u tools/bnrelu_in_lab.py 2>&1 | grep -v amdgpu.ids
echo "-- staged through registers"; timeout -k 10 120 python -u tools/bnrelu_in_lab.py 2>&1 | grep -v amdgpu.ids
bash tools/ab_env.sh bnrreg "SSIP_HALO_DIAG=32" "SSIP_HALO_DIAG=0" 3 || exit 1
