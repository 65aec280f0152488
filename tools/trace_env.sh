# rocprofv3 kernel trace of bench.py under environment settings, one run per
# setting (the program directly after `--`; env applied to rocprofv3 itself).
# usage: bash tools/trace_env.sh <tag> "<envA>" ["<envB>" ...]
set -o pipefail
export TMPDIR=/tmp
tag=$1; shift
i=0
for e in "$@"; do
  o=gpurun_out/tr_$tag/$i
  mkdir -p $o
  env $e timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o -o run -- \
    python bench.py --steps 10 --warmup 5 --no-cpu-baseline > $o/trace.log 2>&1 || { echo "trace $e failed"; tail -5 $o/trace.log; exit 1; }
  echo "$e" > $o/env.txt
  i=$((i+1))
done
