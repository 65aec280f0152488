#!/bin/bash
# Operand-fill ablation of the LDS-DMA conv kernel (timing only, results wrong):
# SSIP_DIAG=0 normal, 1 = A loads dropped, 2 = B loads dropped, 3 = both.
# usage: bash tools/diag_fill.sh <tag> [extra tune_conv args]
set -o pipefail
tag=${1:-diag}; shift
out=gpurun_out/$tag
mkdir -p $out
for d in 0 1 2 3; do
  SSIP_DIAG=$d timeout -k 10 200 python tools/tune_conv.py --no-check --iters 20 --out $out/d$d.json "$@" \
    > $out/d$d.txt 2>&1 || { tail -20 $out/d$d.txt; exit 1; }
  echo "== SSIP_DIAG=$d"; cat $out/d$d.txt
done
