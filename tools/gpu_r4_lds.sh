#!/bin/bash
# GPU box: LDS bank-conflict cycles per kernel (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE), one PMC pass
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/lds
mkdir -p $o
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS --output-format csv -d $o/pmc -o run -- \
  python3 bench.py --steps 3 --warmup 3 --no-cpu-baseline --exec eager > $o/pmc.log 2>&1 || { tail -5 $o/pmc.log; exit 1; }
echo done
