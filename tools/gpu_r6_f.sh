#!/bin/bash
# GPU box (round 6): R50 conv3 BN+ReLU-in per-launch lab, counter names, config-5 A/B.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6f
mkdir -p $o
(rocprofv3 -L 2>/dev/null || true) > $o/counters_all.txt; grep -i -E "MFMA|COEXEC" $o/counters_all.txt | head -30
timeout -k 10 300 python -u tools/inbn_lab.py > $o/inbn_lab.log 2>&1 || { tail -20 $o/inbn_lab.log; exit 1; }
grep -v amdgpu.ids $o/inbn_lab.log
bash tools/ab_env.sh r6f_c5 "SSIP_BNRELU_GLDS=0" "SSIP_BNRELU_GLDS=1" 2 --arch resnet50 --image-size 512 --batch 128 || exit 1
