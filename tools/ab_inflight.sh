# A/B: bench ms/step at host in-flight bounds (SemiStep.max_inflight), alternated runs
set -o pipefail
mkdir -p gpurun_out/inflight
for n in ${@:-0 2 0 2}; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 --max-inflight $n > gpurun_out/inflight/b$n.log 2>&1 || exit 1
  echo "inflight $n: $(tail -1 gpurun_out/inflight/b$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
