#!/bin/bash
# GPU box (round 4): main-loop lab, A/B of the weight-refresh stream default, bench line.
# (SSIP_STEM_MAIN was removed in round 4; its A/B is gone with it.)
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-combo}
mkdir -p $o
timeout -k 10 120 ./tools/lab/gemm_lab 20 > $o/lab.log 2>&1 || { echo lab failed; tail -5 $o/lab.log; exit 1; }
cat $o/lab.log
bash tools/ab_env.sh prep "SSIP_PREP_SIDE=1" "SSIP_PREP_SIDE=0" 3 || exit 1
timeout -k 10 420 python bench.py --cpu-warmup 1 --cpu-steps 3 > $o/bench.log 2>&1 || { echo bench failed; tail -5 $o/bench.log; exit 1; }
tail -1 $o/bench.log
