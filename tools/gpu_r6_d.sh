#!/bin/bash
# GPU box (round 6): step trace with the stagger on (per-stream families), counter list, 16-wave budget wgrad.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6d
mkdir -p $o
(rocprofv3 -L 2>/dev/null || true) | grep -i -E "MFMA|COEXEC|WAIT_ANY|VALU_BUSY" | head -40 > $o/counters.txt
cat $o/counters.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/trace -o run -- \
  python bench.py --steps 10 --warmup 5 --no-cpu-baseline > $o/trace.log 2>&1 || { tail -20 $o/trace.log; exit 1; }
f=$(ls $o/trace/*/run_kernel_trace.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(find $o/trace -name "*kernel_trace.csv" | head -1)
python tools/step_families.py $f > $o/families.txt && head -45 $o/families.txt
python tools/step_streams.py $f > $o/streams.txt && head -12 $o/streams.txt
timeout -k 10 300 python -u tools/wgrad_lab.py --cfg "default;128,128,4,4,2" --budgets 256 > $o/wgrad_lab.log 2>&1 || { tail -20 $o/wgrad_lab.log; exit 1; }
grep -v amdgpu.ids $o/wgrad_lab.log
bash tools/ab_env.sh r6d_wg16 "SSIP_CONV_FORCE=" "SSIP_CONV_FORCE=w,128,128,4,4,2" 3
