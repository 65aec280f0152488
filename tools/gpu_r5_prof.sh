#!/bin/bash
# GPU box (round 5): the bench line plus rocprofv3 passes of exactly the launches
# bench.py's roofline legs time:
#   legs: --profile-leg full / production (single stream, eager, no event timers),
#         kernel trace + stats, and an MFMA-busy PMC pass of each
#   step: kernel trace of the plan-replayed step, FETCH/WRITE PMC passes (eager)
# usage: bash tools/gpu_r5_prof.sh <tag> [extra bench args]
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r5prof}; shift
extra=("$@")
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python bench.py "${extra[@]}" > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log | cut -c1-400
for leg in full production; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/leg_$leg -o run -- \
    python bench.py --profile-leg $leg --steps 3 --warmup 3 "${extra[@]}" > $out/leg_$leg.log 2>&1 || { tail -20 $out/leg_$leg.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY \
    SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $out/mfma_$leg -o run -- \
    python bench.py --profile-leg $leg --steps 2 --warmup 3 "${extra[@]}" > $out/mfma_$leg.log 2>&1 || { tail -20 $out/mfma_$leg.log; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
  python bench.py --steps 10 --warmup 5 --no-cpu-baseline "${extra[@]}" > $out/trace.log 2>&1 || { tail -20 $out/trace.log; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $out/$c -o run -- \
    python bench.py --steps 3 --warmup 3 --no-cpu-baseline --exec eager "${extra[@]}" > $out/$c.log 2>&1 || { tail -20 $out/$c.log; exit 1; }
done
timeout -k 10 300 python bench.py --dtype fp32 --steps 5 --warmup 2 --no-cpu-baseline > $out/bench_fp32.log 2>&1 || { tail -20 $out/bench_fp32.log; exit 1; }
tail -1 $out/bench_fp32.log | cut -c1-400
echo "prof $tag done"
