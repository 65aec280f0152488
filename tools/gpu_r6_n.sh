#!/bin/bash
# GPU box (round 6): the stagger with every LDS read retired before the barrier -- dp2 determinism x3,
# bitwise lab, then the step A/B of the fix.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6n
mkdir -p $o
for i in 1 2 3; do
  timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_gpu_dist.py -k "dp2_bench" > $o/t$i.log 2>&1; rc=$?
  echo "dp2 run $i rc=$rc $(grep -E "AssertionError: |passed|failed" $o/t$i.log | tail -2 | tr '\n' ' ')"
  [ $rc = 0 ] || exit 1
done
timeout -k 10 400 python -u tools/stagger_lab.py --rounds 2 > $o/lab.log 2>&1 || { tail -20 $o/lab.log; exit 1; }
grep -v amdgpu.ids $o/lab.log | tail -8
bash tools/ab_env.sh r6n "SSIP_STAGGER=0" "SSIP_STAGGER=7" 3
