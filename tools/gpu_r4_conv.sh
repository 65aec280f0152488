#!/bin/bash
# GPU box: conv parity tests, the bench line, the per-launch conv breakdown.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-conv}
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_geometry.py tests/test_gpu_conv.py tests/test_gpu_r50_geometry.py tests/test_gpu_fwd_ds.py tests/test_gpu_semi_step.py -x -q --timeout 300 --timeout-method thread > $o/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -2 $o/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python bench.py --cpu-warmup 1 --cpu-steps 3 > $o/bench.log 2>&1 || { echo bench failed; tail -5 $o/bench.log; exit 1; }
tail -1 $o/bench.log
timeout -k 10 300 python tools/conv_breakdown.py > $o/breakdown.log 2>&1 || { echo breakdown failed; tail -5 $o/breakdown.log; exit 1; }
tail -6 $o/breakdown.log
