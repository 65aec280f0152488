#!/bin/bash
# GPU box: conflict-free 64-column MTile swizzle -- wgrad parity, LDS bank conflicts, conv breakdown, step A/B
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/swz
mkdir -p $o
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_halo.py tests/test_gpu_bench_geometry.py tests/test_gpu_c5.py tests/test_gpu_conv.py tests/test_gpu_r50_geometry.py tests/test_gpu_semi_step.py > $o/pytest.log 2>&1 || { tail -20 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
bash tools/gpu_r4_lds.sh
for i in 1 2; do
  SSIP_LIB=ab/libssip_base.so timeout -k 10 300 python tools/conv_breakdown.py > $o/base$i.log 2>&1 || { echo base failed; tail -5 $o/base$i.log; exit 1; }
  timeout -k 10 300 python tools/conv_breakdown.py > $o/new$i.log 2>&1 || { echo new failed; tail -5 $o/new$i.log; exit 1; }
  echo "run $i base: $(grep '^wgrad' $o/base$i.log)  $(tail -1 $o/base$i.log)"
  echo "run $i new:  $(grep '^wgrad' $o/new$i.log)  $(tail -1 $o/new$i.log)"
done
bash tools/ab_worktree.sh swz 3
