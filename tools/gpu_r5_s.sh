#!/bin/bash
# GPU box (round 5): the step boundary's idle time (kernel + memory-copy trace), and the
# trunk's last wgrad at the full grid (SSIP_LAST_WG_FULL) A/B.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5s
mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $o/trace -o run -- \
  python bench.py --steps 10 --warmup 5 --no-cpu-baseline > $o/trace.log 2>&1 || { tail -20 $o/trace.log; exit 1; }
tail -1 $o/trace.log | cut -c1-200
bash tools/ab_env.sh lastwg "SSIP_LAST_WG_FULL=0" "SSIP_LAST_WG_FULL=1" 4 || exit 1
