# A/B of the working tree against a git revision on one box: bench ms/step,
# alternated runs.  Build the baseline first (here, not on the box):
#   git worktree add -f ab_base <rev> && (cd ab_base && python -c "import __graft_entry__ as g; g.build()")
# then on the box: bash tools/ab_worktree.sh <tag> [rounds [extra bench.py args...]]
set -o pipefail
tag=$1; n=${2:-3}
shift $(( $# < 2 ? $# : 2 ))
o=$PWD/gpurun_out/abw_$tag
mkdir -p $o
for i in $(seq 1 $n); do
  for side in base new; do
    if [ $side = base ]; then d=ab_base; else d=.; fi
    (cd $d && timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 "$@" > $o/$side$i.log 2>&1) || { echo "$side$i failed"; tail -5 $o/$side$i.log; exit 1; }
    echo "$side run $i: $(tail -1 $o/$side$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
