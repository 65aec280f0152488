#!/bin/bash
# GPU box (round 6): tile-round quantisation of the layer-2 128x128 launches (1568 tiles on 512 slots at
# batch 256): the same shapes at batch 240 / 245 / 250 / 256 / 262
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6q2
mkdir -p $o
for b in 240 245 250 256 262; do
  timeout -k 10 200 python -u tools/tile_force_lab.py --batch $b --cfg "128,128,4,2,2" --modes fd \
    --shapes l2.3x3,l2.3x3s2 --rounds 2 > $o/b$b.log 2>&1 || { tail -5 $o/b$b.log; exit 1; }
  echo "== batch $b"; grep "default .* us" $o/b$b.log
done
