#!/bin/bash
# GPU box (round 4 calibration): advice-fix tests, vendor-library ceiling on the conv shapes
# (kernel names from a rocprofv3 kernel trace), the bench line.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4cal
mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_semi_step.py -x -q --timeout 200 --timeout-method thread > $o/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -3 $o/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u tools/vendor_ceiling.py > $o/vendor.log 2>&1 || { echo vendor failed; tail -20 $o/vendor.log; exit 1; }
cat $o/vendor.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o vend -- python tools/vendor_ceiling.py --iters 5 > $o/vendor_prof.log 2>&1 || { echo vendor prof failed; tail -5 $o/vendor_prof.log; exit 1; }
timeout -k 10 420 python bench.py > $o/bench.log 2>&1 || { echo bench failed; tail -5 $o/bench.log; exit 1; }
tail -1 $o/bench.log
