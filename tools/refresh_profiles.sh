#!/bin/bash
# GPU box: the bench line, kernel-trace stats of the bench command, and the
# FETCH_SIZE / WRITE_SIZE / MFMA-busy PMC passes (separate runs, eager
# launches so every dispatch is counted; MI355X_MICROARCH.md HBM section).
# usage: bash tools/refresh_profiles.sh <tag> [extra bench.py args, e.g. --arch resnet50 --image-size 512 --batch 128]
#   -> gpurun_out/<tag>/...
# Post-process on the host: tools/prof_summary.py, tools/pmc_traffic.py,
# tools/pmc_mfma.py; copy the summaries into profiles/.
set -o pipefail
export TMPDIR=/tmp
tag=${1:-prof}
shift
extra=("$@")
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python bench.py "${extra[@]}" > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
  python bench.py --steps 10 --warmup 5 --no-cpu-baseline "${extra[@]}" > $out/trace.log 2>&1 || { tail -20 $out/trace.log; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $out/$c -o run -- \
    python bench.py --steps 3 --warmup 3 --no-cpu-baseline --exec eager "${extra[@]}" > $out/$c.log 2>&1 || { tail -20 $out/$c.log; exit 1; }
done
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY \
  SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $out/mfma -o run -- \
  python bench.py --steps 3 --warmup 3 --no-cpu-baseline --exec eager "${extra[@]}" > $out/mfma.log 2>&1 || { tail -20 $out/mfma.log; exit 1; }
echo "refresh $tag done"
