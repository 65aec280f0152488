#!/bin/bash
# GPU box (round 6): the halo epilogue with packed statistics and paired bf16
# conversions -- parity, phase stamps, per-launch and step A/B against HEAD's library (ab_base)
set -o pipefail
export TMPDIR=/tmp
R=$PWD
o=gpurun_out/r6t
mkdir -p $o
BASE=$R/ab_base/semi-supervised-image-processing_amd/ssip/libssip_hip.so
NEW=$R/semi-supervised-image-processing_amd/ssip/libssip_hip.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_halo.py tests/test_gpu_bnrelu_in.py tests/test_gpu_bench_geometry.py tests/test_gpu_eval_fold.py \
  > $o/tests.log 2>&1 || { echo tests failed; tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
timeout -k 10 120 python -u tools/halo_stamp_lab.py --out $o/stamps_new.txt --label new > $o/stamps_new.log 2>&1 || { tail -20 $o/stamps_new.log; exit 1; }
cat $o/stamps_new.txt
SSIP_LIB=$BASE timeout -k 10 120 python -u tools/halo_stamp_lab.py --out $o/stamps_base.txt --label base > $o/stamps_base.log 2>&1 || { tail -20 $o/stamps_base.log; exit 1; }
cat $o/stamps_base.txt
for r in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then L=$BASE; else L=$NEW; fi
    SSIP_LIB=$L timeout -k 10 200 python -u tools/halo_lab.py --diags 0 > $o/halo_${v}_$r.log 2>&1 || { tail -5 $o/halo_${v}_$r.log; exit 1; }
    echo "== $v $r"; grep "diag 0\|residual" $o/halo_${v}_$r.log
  done
done
bash tools/ab_env.sh r6t "SSIP_LIB=$BASE" "SSIP_LIB=$NEW" 3 || exit 1
