#!/bin/bash
# Alternated bench runs of several environment settings on one box.
# usage: bash tools/ab_multi.sh <tag> <rounds> "<env0>" "<env1>" ... [-- extra bench.py args]
set -o pipefail
tag=$1; n=$2; shift 2
envs=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do envs+=("$1"); shift; done
[ "$1" = "--" ] && shift
o=gpurun_out/abm_$tag
mkdir -p $o
for i in $(seq 1 $n); do
  for k in "${!envs[@]}"; do
    e=${envs[$k]}
    env $e timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 "$@" > $o/v$k.$i.log 2>&1 || { echo "v$k.$i failed"; tail -5 $o/v$k.$i.log; exit 1; }
    echo "[$e] run $i: $(tail -1 $o/v$k.$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["sclk"]["mean_mhz"])')"
  done
done
