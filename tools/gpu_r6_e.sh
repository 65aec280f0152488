#!/bin/bash
# GPU box (round 6): BN+ReLU-in on the LDS-DMA ring (R50 conv3 1x1; R18 3x3 opt-in): parity tests,
# config-5 and config-3 step A/Bs; then the step trace (per-stream families) and the 16-wave budget wgrad A/B.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6e
mkdir -p $o
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_bnrelu_in_glds.py tests/test_gpu_semi_step.py -k "glds or r50" > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
grep -E "PASS|FAIL" $o/tests.log
bash tools/ab_env.sh r6e_c5 "SSIP_BNRELU_GLDS=0" "SSIP_BNRELU_GLDS=1" 2 --arch resnet50 --image-size 512 --batch 128 || exit 1
bash tools/ab_env.sh r6e_r18 "SSIP_BNRELU_GLDS=1" "SSIP_BNRELU_GLDS=3" 3 || exit 1
bash tools/ab_env.sh r6e_c5b "SSIP_BNRELU_GLDS=1" "SSIP_BNRELU_GLDS=3" 2 --arch resnet50 --image-size 512 --batch 128 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/trace -o run -- \
  python bench.py --steps 10 --warmup 5 --no-cpu-baseline > $o/trace.log 2>&1 || { tail -20 $o/trace.log; exit 1; }
f=$(find $o/trace -name "*kernel_trace.csv" | head -1)
python tools/step_families.py $f > $o/families.txt && head -50 $o/families.txt
python tools/step_streams.py $f > $o/streams.txt && head -12 $o/streams.txt
