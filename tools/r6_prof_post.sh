#!/bin/bash
# Host side after tools/gpu_r6_prof.sh <tag>: copy the one-lease profile summaries into profiles/.
# usage: bash tools/r6_prof_post.sh <tag> [prefix (default r6)] [workload key for the PMC traffic file]
set -e
tag=${1:-r6prof}; pre=${2:-r6}
key=${3:-semi_consistency_resnet18_224 bs256 labeled128 bf16}
src=gpurun_out/$tag
tail -1 $src/bench.log > profiles/${pre}_prof_bench_line.json
tf=$(python3 -c "import json; print(json.loads(open('$src/bench.log').read().strip().splitlines()[-1])['config']['gflop_per_step_per_gpu'] / 1000)")
for leg in full production production_s0; do
  # recomputed here from the trace with the line's own TFLOP per step (the box-side pass of round-6's
  # first config-5 lease used the R18 default)
  f=$(find $src/leg_$leg -name "*kernel_trace.csv" 2>/dev/null | head -1)
  if [ -n "$f" ]; then
    mhz=$(python3 -c "import json; print(json.load(open('$src/sclk_$leg.json'))['sclk']['mean_mhz'])")
    lab="leg $leg (SCLK $mhz MHz)"; [ $leg = production_s0 ] && lab="leg production, SSIP_STAGGER=0 (SCLK $mhz MHz)"
    python3 tools/roofline_from_trace.py $f --tflop $tf --label "$lab" --out profiles/${pre}_roofline_leg_$leg.txt | head -2
  fi
  [ -f $src/mfma_busy_leg_$leg.txt ] && cp $src/mfma_busy_leg_$leg.txt profiles/${pre}_mfma_busy_leg_$leg.txt
done
python3 - "$src" "$pre" <<'EOF'
import glob, json, sys
src, pre = sys.argv[1], sys.argv[2]
out = {}
for f in sorted(glob.glob(f"{src}/sclk_*.json")):
    out[f.split("/")[-1][5:-5]] = json.load(open(f))["sclk"]
json.dump(out, open(f"profiles/{pre}_prof_sclk.json", "w"), indent=1)
print("sclk per pass:", {k: v.get("mean_mhz") for k, v in out.items()})
EOF
for leg in full production; do
  f=$(find $src/leg_$leg -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] && cp $f profiles/${pre}_leg_${leg}_kernel_stats.csv
done
fe=$(find $src/FETCH_SIZE -name "*counter_collection.csv" | head -1)
wr=$(find $src/WRITE_SIZE -name "*counter_collection.csv" | head -1)
python3 tools/pmc_traffic.py $fe $wr profiles/${pre}_pmc_traffic.json "$key"
ls -la profiles/${pre}_*
