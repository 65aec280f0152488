# A/B of environment settings on one box: bench ms/step, alternated runs.
# usage: bash tools/ab_env.sh <tag> "<envA>" "<envB>" [rounds [extra bench.py args...]]
#   e.g. bash tools/ab_env.sh fuse "SSIP_FUSE_BN_BWD=0" "SSIP_FUSE_BN_BWD=1" 3
set -o pipefail
tag=$1; a=$2; b=$3; n=${4:-2}
shift $(( $# < 4 ? $# : 4 ))
o=gpurun_out/ab_$tag
mkdir -p $o
for i in $(seq 1 $n); do
  for side in A B; do
    if [ $side = A ]; then e=$a; else e=$b; fi
    env $e timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 "$@" > $o/$side$i.log 2>&1 || { echo "$side$i failed"; tail -5 $o/$side$i.log; exit 1; }
    echo "$side [$e] run $i: $(tail -1 $o/$side$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
