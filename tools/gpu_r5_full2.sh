#!/bin/bash
# GPU box (round 5): the whole GPU suite + smoke on the final code.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5full4
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu > $o/tests.log 2>&1 || { echo tests failed; tail -40 $o/tests.log; exit 1; }
tail -3 $o/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.log 2>&1 || { tail -20 $o/smoke.log; exit 1; }
tail -2 $o/smoke.log
