#!/bin/bash
# GPU box (round 6): isolate the dp2 bench-geometry gradient mismatch (defaults vs SSIP_WGRAD_BIG=0 vs SSIP_STAGGER=0).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6m
mkdir -p $o
for e in "SSIP_WGRAD_BIG=0" "SSIP_STAGGER=0" "SSIP_X=1"; do
  env $e timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_gpu_dist.py -k "dp2_bench" > $o/t_$e.log 2>&1
  echo "[$e] rc=$? $(grep -E "AssertionError: |passed|failed" $o/t_$e.log | tail -2 | tr '\n' ' ')"
done
