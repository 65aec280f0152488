#!/bin/bash
# GPU box: kernel-trace stats of the bench command + FETCH_SIZE / WRITE_SIZE
# PMC passes (separate runs, eager launches so every dispatch is counted).
# Outputs under gpurun_out/prof_r1/; post-process with tools/prof_summary.py
# and tools/pmc_traffic.py, then copy the summaries into profiles/.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/prof_r1b
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
  python bench.py --steps 10 --warmup 5 --no-cpu-baseline > $out/trace.log 2>&1 || { tail -20 $out/trace.log; exit 1; }
tail -1 $out/trace.log
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $out/$c -o run -- \
    python bench.py --steps 3 --warmup 3 --no-cpu-baseline --eager > $out/$c.log 2>&1 || { tail -20 $out/$c.log; exit 1; }
done
find $out -name "*.csv" | head -20
