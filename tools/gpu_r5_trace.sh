#!/bin/bash
# GPU box: kernel trace of the plan-replayed bench step (current defaults).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r5t}
mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/trace -o run -- \
  python bench.py --steps 10 --warmup 5 --no-cpu-baseline > $o/trace.log 2>&1 || { tail -20 $o/trace.log; exit 1; }
tail -1 $o/trace.log | cut -c1-200
