#!/bin/bash
# GPU box (round 5), in two calls (each within gpurun's 20 minutes):
#   part line: the bench line (with the CPU baseline), the fp32 step line, a kernel trace of the
#              plan-replayed step
#   part legs: rocprofv3 passes of exactly the launches bench.py's roofline legs time (VERDICT r4
#              item 1): --profile-leg full / production (single stream, eager, no event timers),
#              kernel trace + stats and an MFMA-busy PMC pass of each; FETCH/WRITE PMC passes (eager)
# usage: bash tools/gpu_r5_prof.sh <tag> line|legs [extra bench args]
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r5prof}; part=${2:-line}; shift 2
extra=("$@")
out=gpurun_out/$tag
mkdir -p $out
if [ $part = line ]; then
  timeout -k 10 600 python bench.py "${extra[@]}" > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
  tail -1 $out/bench.log | cut -c1-400
  timeout -k 10 300 python bench.py --dtype fp32 --steps 5 --warmup 2 --no-cpu-baseline > $out/bench_fp32.log 2>&1 || { tail -20 $out/bench_fp32.log; exit 1; }
  tail -1 $out/bench_fp32.log | cut -c1-400
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
    python bench.py --steps 10 --warmup 5 --no-cpu-baseline "${extra[@]}" > $out/trace.log 2>&1 || { tail -20 $out/trace.log; exit 1; }
else
  for leg in full production; do
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/leg_$leg -o run -- \
      python bench.py --profile-leg $leg --steps 3 --warmup 3 "${extra[@]}" > $out/leg_$leg.log 2>&1 || { tail -20 $out/leg_$leg.log; exit 1; }
    timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY \
      SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $out/mfma_$leg -o run -- \
      python bench.py --profile-leg $leg --steps 2 --warmup 3 "${extra[@]}" > $out/mfma_$leg.log 2>&1 || { tail -20 $out/mfma_$leg.log; exit 1; }
  done
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $out/$c -o run -- \
      python bench.py --steps 3 --warmup 3 --no-cpu-baseline --exec eager "${extra[@]}" > $out/$c.log 2>&1 || { tail -20 $out/$c.log; exit 1; }
  done
fi
du -sh $out
echo "prof $tag $part done"
