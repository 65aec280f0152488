#!/bin/bash
# GPU box (round 6): the whole -m gpu suite + smoke, as the driver runs them.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r6full}
mkdir -p $o
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 400 --timeout-method thread > $o/tests.log 2>&1; rc=$?
tail -5 $o/tests.log
grep -E "FAILED|Error" $o/tests.log | head -20
[ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { tail -20 $o/smoke.log; exit 1; }
tail -2 $o/smoke.log
