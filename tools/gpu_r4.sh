#!/bin/bash
# GPU box (round 4): full GPU test suite, smoke, bench line.
# usage: bash tools/gpu_r4.sh <tag> [pytest -k expr] [bench args...]
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r4}
o=gpurun_out/$tag
mkdir -p $o
if [ -n "$2" ]; then k=(-k "$2"); else k=(); fi
shift $(( $# < 2 ? $# : 2 ))
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${k[@]}" > $o/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -5 $o/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { echo smoke failed; tail -5 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
timeout -k 10 420 python bench.py --cpu-warmup 1 --cpu-steps 3 "$@" > $o/bench.log 2>&1 || { echo bench failed; tail -5 $o/bench.log; exit 1; }
tail -1 $o/bench.log
if [ -x tools/lab/gemm_lab ] && [ -n "$R4_LAB" ]; then
  timeout -k 10 120 ./tools/lab/gemm_lab 20 > $o/lab.log 2>&1 || { echo lab failed; tail -5 $o/lab.log; exit 1; }
  cat $o/lab.log
fi
