#!/bin/bash
# GPU box (round 5): deeper-ring fwd/dgrad tiles (3-stage 256x128 / 128x128) on layers 2-4.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5l
mkdir -p $o
timeout -k 10 600 python -u tools/tune_conv.py --modes fd --iters 20 --shapes l2.3x3,l2.3x3s2,l3.3x3,l3.3x3s2,l4.3x3,l4.3x3s2 \
  --fd "128,128,4,2,2;256,256,4,2,2;128,128,4,4,3;256,128,4,2,3;256,128,4,4,3;128,128,4,2,3" --out $o/tune.json \
  > $o/tune.log 2>&1 || { tail -20 $o/tune.log; exit 1; }
grep -v amdgpu.ids $o/tune.log
python - <<'PY'
import json
for r in json.load(open("gpurun_out/r5l/tune.json")):
    print(r["shape"], r["mode"], round(r["default_us"],1), {k: (round(v,1) if isinstance(v,float) else v) for k,v in r["cfg"].items()})
PY
