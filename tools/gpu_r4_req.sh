#!/bin/bash
# GPU box: L1 -> L2 request counts per kernel (coalescing audit), one PMC pass
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/req
mkdir -p $o
timeout -s KILL 240 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum --output-format csv -d $o/pmc -o run -- \
  python3 bench.py --steps 3 --warmup 3 --no-cpu-baseline --exec eager > $o/pmc.log 2>&1 || { tail -5 $o/pmc.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/w -o run -- \
  python3 bench.py --steps 3 --warmup 3 --no-cpu-baseline --exec eager > $o/w.log 2>&1 || { tail -5 $o/w.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/f -o run -- \
  python3 bench.py --steps 3 --warmup 3 --no-cpu-baseline --exec eager > $o/f.log 2>&1 || { tail -5 $o/f.log; exit 1; }
echo done
