#!/bin/bash
# GPU box (round 5): one main->side event per block (SSIP_WGRAD_BATCH) and one-wave finalize
# workgroups (SSIP_FIN64): step parity tests, then alternated step A/Bs, then a trace.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5f
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_semi_step.py tests/test_gpu_rccl.py tests/test_gpu_resnet.py \
  > $o/tests.log 2>&1 || { echo tests failed; tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
bash tools/ab_env.sh wbatch "SSIP_WGRAD_BATCH=0" "SSIP_WGRAD_BATCH=1" 3 || exit 1
bash tools/ab_env.sh fin64 "SSIP_FIN64=0" "SSIP_FIN64=1" 3 || exit 1
SSIP_FIN64=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/trace -o run -- \
  python bench.py --steps 10 --warmup 5 --no-cpu-baseline > $o/trace.log 2>&1 || { tail -20 $o/trace.log; exit 1; }
echo done
