#!/bin/bash
# GPU box (round 4 calibration): vendor-library ceiling on the conv shapes + the bench line.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4cal
mkdir -p $o
timeout -k 10 300 python -u tools/vendor_ceiling.py > $o/vendor.log 2>&1 || { echo vendor failed; tail -20 $o/vendor.log; exit 1; }
cat $o/vendor.log
timeout -k 10 420 python bench.py > $o/bench.log 2>&1 || { echo bench failed; tail -5 $o/bench.log; exit 1; }
tail -1 $o/bench.log
