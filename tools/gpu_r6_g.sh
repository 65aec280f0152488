#!/bin/bash
# GPU box (round 6): tile choices with the stagger on -- ResNet-50 1x1 convs (config 5), ResNet-18 layer-4
# 256x256 and the weak forward's batch-128 tiles; budget wgrad tiles.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6g
mkdir -p $o
timeout -k 10 400 python -u tools/tile_force_lab.py --r50 --batch 128 --cfg "128,128,4,2,2;256,256,4,2,2;128,64,4,2,2" \
  > $o/r50_tiles.log 2>&1 || { tail -20 $o/r50_tiles.log; exit 1; }
grep -v amdgpu.ids $o/r50_tiles.log
timeout -k 10 300 python -u tools/tile_force_lab.py --shapes l4.3x3s2,l4.3x3,l3.3x3s2 --cfg "256,256,4,2,2;128,128,4,4,3" \
  > $o/r18_tiles.log 2>&1 || { tail -20 $o/r18_tiles.log; exit 1; }
grep -v amdgpu.ids $o/r18_tiles.log
timeout -k 10 300 python -u tools/tile_force_lab.py --batch 128 --modes f --shapes l2.3x3s2,l2.3x3,l3.3x3s2,l3.3x3,l4.3x3s2,l4.3x3 \
  --cfg "128,128,4,2,2;128,128,4,4,3;256,256,4,2,2" > $o/weak_tiles.log 2>&1 || { tail -20 $o/weak_tiles.log; exit 1; }
grep -v amdgpu.ids $o/weak_tiles.log
timeout -k 10 300 python -u tools/wgrad_lab.py --cfg "default;256,256,4,2,2;128,128,4,4,2;256,256,4,4,2" --budgets 256 \
  > $o/wgrad_lab.log 2>&1 || { tail -20 $o/wgrad_lab.log; exit 1; }
grep -v amdgpu.ids $o/wgrad_lab.log
