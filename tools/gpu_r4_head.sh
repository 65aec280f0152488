#!/bin/bash
# GPU box: head-kernel parity and step A/B vs ab_base
set -o pipefail
o=gpurun_out/head
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_semi_step.py > $o/pytest.log 2>&1 || { tail -20 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
bash tools/ab_worktree.sh head 3
