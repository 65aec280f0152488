#!/bin/bash
# GPU box: selected GPU test files, then the bench line and the conv breakdown.
# usage: bash tools/gpu_quick.sh <tag> <test files...>
set -o pipefail
export TMPDIR=/tmp
tag=$1; shift
o=gpurun_out/$tag
mkdir -p $o
timeout -k 10 600 python -u -m pytest "$@" -x -v --timeout 200 --timeout-method thread > $o/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "passed|failed|error" $o/pytest.log | tail -3
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 420 python bench.py > $o/bench.log 2>&1 || { echo bench failed; tail -5 $o/bench.log; exit 1; }
tail -1 $o/bench.log
timeout -k 10 300 python tools/conv_breakdown.py > $o/breakdown.log 2>&1 || { echo breakdown failed; tail -5 $o/breakdown.log; exit 1; }
tail -4 $o/breakdown.log
