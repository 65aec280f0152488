#!/bin/bash
# GPU box (round 6): halo epilogue stagger (lab + step A/B), wide fwd/dgrad tiles, 3-stage budget wgrad,
# the real-data N1 test and the all-reduce overlap test.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6c
mkdir -p $o
timeout -k 10 300 python -u tools/halo_stagger_lab.py > $o/halo_lab.log 2>&1 || { tail -20 $o/halo_lab.log; exit 1; }
grep -v amdgpu.ids $o/halo_lab.log
timeout -k 10 300 python -u tools/tile_force_lab.py > $o/tile_lab.log 2>&1 || { tail -20 $o/tile_lab.log; exit 1; }
grep -v amdgpu.ids $o/tile_lab.log
timeout -k 10 300 python -u tools/wgrad_lab.py --cfg "default;128,128,4,2,3" --budgets 0,256 > $o/wgrad_lab.log 2>&1 || { tail -20 $o/wgrad_lab.log; exit 1; }
grep -v amdgpu.ids $o/wgrad_lab.log
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_real_data.py tests/test_gpu_dist.py -k "real or overlap" > $o/tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|max dP|max \||flips|_loss|Error|baseline_" $o/tests.log | head -60
[ $rc = 0 ] || exit $rc
bash tools/ab_env.sh r6c_halo "SSIP_HALO_STAGGER=0" "SSIP_HALO_STAGGER=1" 3
