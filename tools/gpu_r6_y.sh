#!/bin/bash
# GPU box (round 6): the SB halo form (32-column panels, two 4-wave workgroups per CU) -- parity,
# per-launch lab and step A/B against the 8-wave form
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6y
mkdir -p $o
SSIP_HALO_SB=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -k "not partial_tiles_is_workgroup_count" \
  tests/test_gpu_halo.py tests/test_gpu_bnrelu_in.py tests/test_gpu_eval_fold.py tests/test_gpu_semi_step.py \
  > $o/tests.log 2>&1 || { echo tests failed; tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
for r in 1 2; do
  for v in 0 1; do
    SSIP_HALO_SB=$v timeout -k 10 200 python -u tools/halo_lab.py --diags 0 > $o/halo_${v}_$r.log 2>&1 || { tail -5 $o/halo_${v}_$r.log; exit 1; }
    echo "== SB=$v $r"; grep "batch\|diag 0\|residual" $o/halo_${v}_$r.log
  done
done
bash tools/ab_env.sh r6y "SSIP_HALO_SB=0" "SSIP_HALO_SB=1" 3 || exit 1
