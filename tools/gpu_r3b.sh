#!/bin/bash
# GPU box: selected GPU tests, bench line, rocprofv3 kernel trace of the bench (timeline)
set -o pipefail
export TMPDIR=/tmp
tag=$1; shift
o=gpurun_out/$tag
mkdir -p $o
timeout -k 10 900 python -u -m pytest "$@" -x -v --timeout 300 --timeout-method thread > $o/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "passed|failed|error" $o/pytest.log | tail -3
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 420 python bench.py --no-cpu-baseline > $o/bench.log 2>&1 || { echo bench failed; tail -5 $o/bench.log; exit 1; }
tail -1 $o/bench.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace -o run -- \
  python bench.py --steps 10 --warmup 5 --no-cpu-baseline > $o/trace.log 2>&1 || { echo trace failed; tail -5 $o/trace.log; exit 1; }
f=$(find $o/trace -name "*kernel_trace.csv" | head -1)
python tools/step_streams.py $f > $o/streams.txt 2>&1; head -30 $o/streams.txt
