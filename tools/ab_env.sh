#!/bin/bash
# A/B of an environment setting in whole bench steps, alternated on one box.
# usage: bash tools/ab_env.sh <tag> <rounds> "<A env assignments>" "<B env assignments>" [extra bench args]
set -o pipefail
tag=$1; rounds=$2; ea=$3; eb=$4; shift 4
out=gpurun_out/$tag
mkdir -p $out
for i in $(seq 1 $rounds); do
  env $ea timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 "$@" > $out/a$i.log 2>&1 || { tail -5 $out/a$i.log; exit 1; }
  env $eb timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 "$@" > $out/b$i.log 2>&1 || { tail -5 $out/b$i.log; exit 1; }
done
for f in $out/a*.log $out/b*.log; do echo $f $(grep -o '"ms_per_step": [0-9.]*' $f); done
