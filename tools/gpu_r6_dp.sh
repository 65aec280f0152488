#!/bin/bash
# GPU box (round 6): the driver's N>1 bench command rehearsed with 2 ranks sharing the one GPU over gloo
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6dp
mkdir -p $o
SSIP_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > $o/bench2.log 2>&1 \
  || { tail -30 $o/bench2.log; exit 1; }
grep '^{' $o/bench2.log | cut -c1-400
