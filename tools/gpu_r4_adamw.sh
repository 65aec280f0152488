#!/bin/bash
# GPU box: AdamW alone, its parity tests, the step tests, whole-step A/B vs ab_base
set -o pipefail
o=gpurun_out/adamw
mkdir -p $o
timeout -k 10 120 python tools/time_adamw.py > $o/time.log 2>&1 || { tail -5 $o/time.log; exit 1; }
cat $o/time.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_semi_step.py tests/test_gpu_pipeline.py > $o/pytest.log 2>&1 || { tail -20 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
bash tools/ab_worktree.sh adamw 3
