#!/bin/bash
# GPU box (round 5): the whole -m gpu suite and smoke(), as the driver runs them.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5full
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $o/pytest.log 2>&1
rc=$?
tail -5 $o/pytest.log
[ $rc -eq 0 ] || { grep -n "FAILED\|Error\|assert" $o/pytest.log | head -30; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { tail -20 $o/smoke.log; exit 1; }
tail -2 $o/smoke.log
