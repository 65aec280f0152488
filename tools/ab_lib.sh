#!/bin/bash
# A/B of two library builds in whole bench steps, alternated on one box:
# A = ab/libssip_base.so (built from the base commit), B = the in-tree build.
# usage: bash tools/ab_lib.sh <tag> [rounds] [extra bench args]
set -o pipefail
tag=${1:-ab}; rounds=${2:-3}; shift 2
out=gpurun_out/$tag
mkdir -p $out
for i in $(seq 1 $rounds); do
  SSIP_LIB=ab/libssip_base.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 "$@" > $out/a$i.log 2>&1 || { tail -5 $out/a$i.log; exit 1; }
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 "$@" > $out/b$i.log 2>&1 || { tail -5 $out/b$i.log; exit 1; }
done
for f in $out/a*.log $out/b*.log; do echo $f $(grep -o '"ms_per_step": [0-9.]*' $f); done
