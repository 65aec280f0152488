#!/bin/bash
# GPU-box cycle (round 2).  usage: bash tools/gpu_r2.sh <tag> <stage>...
# stages: tests | tests:<pytest -k expr> | bench | bench:<extra args> | trace | mfma | fetch | write
# Every GPU step runs under its own timeout; the script stops at the first failure.
set -o pipefail
tag=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
out=gpurun_out/$tag
mkdir -p $out
nb=0
for st in "$@"; do
  case $st in
    tests|tests:*)
      k=${st#tests}; k=${k#:}
      timeout -k 10 780 python -u -m pytest tests -m gpu -v --maxfail=25 --timeout 240 --timeout-method thread \
        ${k:+-k "$k"} > $out/tests.log 2>&1
      rc=$?; tail -3 $out/tests.log; grep -E "FAILED|ERROR" $out/tests.log | head -30
      [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc   # 1 = test failures (keep going), else abort
      ;;
    bench|bench:*)
      a=${st#bench}; a=${a#:}; nb=$((nb+1))
      timeout -k 10 420 python bench.py $a > $out/bench$nb.log 2>&1 || { tail -20 $out/bench$nb.log; exit 1; }
      tail -1 $out/bench$nb.log
      ;;
    trace)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
        python bench.py --steps 10 --warmup 5 --no-cpu-baseline > $out/trace.log 2>&1 || { tail -20 $out/trace.log; exit 1; }
      tail -1 $out/trace.log
      ;;
    mfma)
      timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY \
        SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $out/mfma -o run -- \
        python bench.py --steps 3 --warmup 3 --no-cpu-baseline > $out/mfma.log 2>&1 || { tail -20 $out/mfma.log; exit 1; }
      tail -1 $out/mfma.log
      ;;
    fetch|write)
      c=FETCH_SIZE; [ $st = write ] && c=WRITE_SIZE
      timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $out/$c -o run -- \
        python bench.py --steps 3 --warmup 3 --no-cpu-baseline > $out/$c.log 2>&1 || { tail -20 $out/$c.log; exit 1; }
      tail -1 $out/$c.log
      ;;
    py:*)
      # an arbitrary python tool: py:<script> [args] (timeout 300)
      c=${st#py:}
      timeout -k 10 300 python $c > $out/py_$(basename ${c%% *} .py).log 2>&1 || { tail -20 $out/py_$(basename ${c%% *} .py).log; exit 1; }
      tail -5 $out/py_$(basename ${c%% *} .py).log
      ;;
    *) echo "unknown stage $st"; exit 2 ;;
  esac
done
echo "gpu_r2 $tag done"
