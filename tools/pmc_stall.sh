#!/bin/bash
# Stall breakdown of single conv kernels: one rocprofv3 --pmc pass per shape.
# usage: bash tools/pmc_stall.sh <tag> "<shape> <mode>" ...
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for sm in "$@"; do
  set -- $sm
  out=$R/gpurun_out/${tag}_$1_$2
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS \
    -d $out -o pmc -- python3 $R/tools/one_conv.py $1 $2 10 > $out.log 2>&1 || { tail -5 $out.log; exit 1; }
done
echo pmc done
