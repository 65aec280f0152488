#!/bin/bash
# GPU-box cycle: parity tests, bench, kernel trace of a short bench.
# usage: bash tools/gpu_cycle.sh <tag> [tests|notests]
set -o pipefail
tag=${1:-cycle}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${2:-tests}" = "tests" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
  tail -2 gpurun_out/${tag}_tests.log
fi
timeout -k 10 240 python bench.py > gpurun_out/${tag}_bench.log 2>&1 || { tail -20 gpurun_out/${tag}_bench.log; exit 1; }
tail -1 gpurun_out/${tag}_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run -- \
  python bench.py --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/${tag}_prof.log 2>&1 || { tail -20 gpurun_out/${tag}_prof.log; exit 1; }
echo cycle done
