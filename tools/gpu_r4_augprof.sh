#!/bin/bash
# GPU box: kernel-trace stats of a short bench, base library vs in-tree (augment kernel timing)
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/augprof
mkdir -p $o
SSIP_LIB=ab/libssip_base.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/base -o run -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 > $o/base.log 2>&1 || { tail -5 $o/base.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/new -o run -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 > $o/new.log 2>&1 || { tail -5 $o/new.log; exit 1; }
for s in base new; do f=$(find $o/$s -name "run_kernel_stats.csv" | head -1); echo "$s: $(grep -iE "${PAT:-augment}" $f | cut -c1-200)"; done
