#!/bin/bash
# GPU box (round 5): step boundary with copy-ahead (kernel + memory-copy trace), more A/B runs.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5ac
mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $o/trace -o run -- \
  python bench.py --steps 10 --warmup 5 --no-cpu-baseline > $o/trace.log 2>&1 || { tail -20 $o/trace.log; exit 1; }
bash tools/ab_env.sh cpahead2 "SSIP_COPY_AHEAD=0" "SSIP_COPY_AHEAD=1" 5 || exit 1
