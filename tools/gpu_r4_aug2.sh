#!/bin/bash
# GPU box: augment with the rows' source loads issued ahead -- bit-exactness, kernel time, step A/B
set -o pipefail
o=gpurun_out/aug2
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_augment.py tests/test_gpu_semi_step.py > $o/pytest.log 2>&1 || { tail -20 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
bash tools/gpu_r4_augprof.sh
bash tools/ab_worktree.sh aug2 3
