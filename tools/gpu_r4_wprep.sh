#!/bin/bash
# GPU box: weight refresh with all loads in flight -- parity (engine + eval fold), kernel time, step A/B
set -o pipefail
o=gpurun_out/wprep
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_semi_step.py tests/test_gpu_eval_fold.py tests/test_gpu_bench_geometry.py > $o/pytest.log 2>&1 || { tail -20 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
PAT=weight_prep bash tools/gpu_r4_augprof.sh
bash tools/ab_worktree.sh wprep 3
