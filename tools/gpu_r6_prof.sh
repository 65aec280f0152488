#!/bin/bash
# GPU box (round 6), ONE lease: the bench line and rocprofv3 traces of exactly
# its two roofline legs on the same box, each leg recording its own SCLK (bench.py --sclk-out), the
# MFMA-busy / wave-state PMC pass per leg normalised by that SCLK, and the conv-family PMC traffic.
# usage: bash tools/gpu_r6_prof.sh <tag> [extra bench args]
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r6prof}; shift
extra=("$@")
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 python bench.py --no-cpu-baseline "${extra[@]}" > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log | cut -c1-300
# the step's conv-family TFLOP from the line itself (R18 3.1895, R50 512^2 18.975)
tf=$(python3 -c "import json; print(json.loads(open('$out/bench.log').read().strip().splitlines()[-1])['config']['gflop_per_step_per_gpu'] / 1000)")
for leg in full production; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/leg_$leg -o run -- \
    python bench.py --profile-leg $leg --steps 3 --warmup 3 --sclk-out $out/sclk_$leg.json "${extra[@]}" \
    > $out/leg_$leg.log 2>&1 || { tail -20 $out/leg_$leg.log; exit 1; }
  f=$(find $out/leg_$leg -name "*kernel_trace.csv" | head -1)
  mhz=$(python3 -c "import json; print(json.load(open('$out/sclk_$leg.json'))['sclk']['mean_mhz'])")
  python3 tools/roofline_from_trace.py $f --tflop $tf --label "leg $leg (SCLK $mhz MHz)" --out $out/roofline_leg_$leg.txt | head -3
  timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY \
    SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE --output-format csv \
    -d $out/mfma_$leg -o run -- \
    python bench.py --profile-leg $leg --steps 2 --warmup 3 --sclk-out $out/sclk_mfma_$leg.json "${extra[@]}" \
    > $out/mfma_$leg.log 2>&1 || { tail -20 $out/mfma_$leg.log; exit 1; }
  f=$(find $out/mfma_$leg -name "*counter_collection.csv" | head -1)
  mhz2=$(python3 -c "import json; print(json.load(open('$out/sclk_mfma_$leg.json'))['sclk']['mean_mhz'])")
  python3 tools/pmc_mfma.py $f $out/mfma_busy_leg_$leg.txt --sclk-mhz $mhz2 | head -12
done
# the stagger's before/after on the same box: the production leg traced and counted
# with SSIP_STAGGER=0
SSIP_STAGGER=0 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/leg_production_s0 -o run -- \
  python bench.py --profile-leg production --steps 3 --warmup 3 --sclk-out $out/sclk_production_s0.json "${extra[@]}" \
  > $out/leg_production_s0.log 2>&1 || { tail -20 $out/leg_production_s0.log; exit 1; }
f=$(find $out/leg_production_s0 -name "*kernel_trace.csv" | head -1)
mhz=$(python3 -c "import json; print(json.load(open('$out/sclk_production_s0.json'))['sclk']['mean_mhz'])")
python3 tools/roofline_from_trace.py $f --tflop $tf --label "leg production, SSIP_STAGGER=0 (SCLK $mhz MHz)" \
  --out $out/roofline_leg_production_s0.txt | head -3
SSIP_STAGGER=0 timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY \
  SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE --output-format csv \
  -d $out/mfma_production_s0 -o run -- \
  python bench.py --profile-leg production --steps 2 --warmup 3 --sclk-out $out/sclk_mfma_production_s0.json "${extra[@]}" \
  > $out/mfma_production_s0.log 2>&1 || { tail -20 $out/mfma_production_s0.log; exit 1; }
f=$(find $out/mfma_production_s0 -name "*counter_collection.csv" | head -1)
mhz2=$(python3 -c "import json; print(json.load(open('$out/sclk_mfma_production_s0.json'))['sclk']['mean_mhz'])")
python3 tools/pmc_mfma.py $f $out/mfma_busy_leg_production_s0.txt --sclk-mhz $mhz2 | head -12
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $out/$c -o run -- \
    python bench.py --steps 3 --warmup 3 --no-cpu-baseline --exec eager "${extra[@]}" > $out/$c.log 2>&1 || { tail -20 $out/$c.log; exit 1; }
done
du -sh $out
echo "prof $tag done"
