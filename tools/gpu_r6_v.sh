#!/bin/bash
# GPU box (round 6): step trace under the round-6 defaults -- per-stream kernel families and idle time
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6v
mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/trace -o run -- \
  python bench.py --steps 10 --warmup 5 --no-cpu-baseline > $o/trace.log 2>&1 || { tail -20 $o/trace.log; exit 1; }
f=$(find $o/trace -name "*kernel_trace.csv" | head -1)
python tools/step_families.py $f > $o/families.txt && cat $o/families.txt
python tools/step_streams.py $f > $o/streams.txt && cat $o/streams.txt
