# rocprofv3 kernel traces of bench.py for the baseline worktree (ab_base) and
# the working tree, for tools/step_families.py / side-by-side sequences.
# usage: bash tools/trace_ab.sh <tag>
set -o pipefail
export TMPDIR=/tmp
tag=$1
R=$PWD
for side in base new; do
  if [ $side = base ]; then d=ab_base; else d=.; fi
  o=$R/gpurun_out/tra_$tag/$side
  mkdir -p $o
  (cd $d && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o -o run -- \
    python bench.py --steps 10 --warmup 5 --no-cpu-baseline > $o/trace.log 2>&1) || { echo "trace $side failed"; tail -5 $o/trace.log; exit 1; }
done
