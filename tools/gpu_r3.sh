#!/bin/bash
# GPU box: round-3 check -- GPU tests, smoke, bench line, conv breakdown.
# usage: bash tools/gpu_r3.sh <tag> [pytest -k expr]
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r3}
o=gpurun_out/$tag
mkdir -p $o
if [ -n "$2" ]; then k=(-k "$2"); else k=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${k[@]}" > $o/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -3 $o/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { echo smoke failed; tail -5 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
timeout -k 10 420 python bench.py > $o/bench.log 2>&1 || { echo bench failed; tail -5 $o/bench.log; exit 1; }
tail -1 $o/bench.log
timeout -k 10 300 python tools/conv_breakdown.py > $o/breakdown.log 2>&1 || { echo breakdown failed; exit 1; }
tail -4 $o/breakdown.log
