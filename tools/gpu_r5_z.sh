#!/bin/bash
# GPU box (round 5): BN+ReLU-in convs with the lane's scale / shift hoisted: parity, lab (new vs the
# previous library abtmp/libssip_old.so), step A/B.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5z
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_bnrelu_in.py > $o/tests.log 2>&1 || { echo tests failed; tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
echo "-- previous"; SSIP_LIB=$PWD/abtmp/libssip_old.so timeout -k 10 120 python -u tools/bnrelu_in_lab.py 2>&1 | grep -v amdgpu.ids
echo "-- hoisted"; timeout -k 10 120 python -u tools/bnrelu_in_lab.py 2>&1 | grep -v amdgpu.ids
bash tools/ab_env.sh bnrhoist "SSIP_LIB=$PWD/abtmp/libssip_old.so" "SSIP_NEW=1" 3 || exit 1
