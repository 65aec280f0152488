#!/bin/bash
# GPU box (round 5): plan replay records each cross-stream event as the stop event of the
# launch before it (SSIP_PLAN_MARKERS=1: separate marker packets, as before): parity of the
# plan / graph / eager steps, alternated step A/B, then a trace of the new default.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5g
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_semi_step.py tests/test_gpu_rccl.py tests/test_gpu_resnet.py tests/test_gpu_dist.py \
  > $o/tests.log 2>&1 || { echo tests failed; tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
bash tools/ab_env.sh markers "SSIP_PLAN_MARKERS=1" "SSIP_PLAN_MARKERS_UNSET=1" 3 || exit 1
bash tools/ab_env.sh fin64c "SSIP_FIN64=0" "SSIP_FIN64=1" 2 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/trace -o run -- \
  python bench.py --steps 10 --warmup 5 --no-cpu-baseline > $o/trace.log 2>&1 || { tail -20 $o/trace.log; exit 1; }
echo done
