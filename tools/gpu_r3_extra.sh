#!/bin/bash
# Round-3 extra evidence on the GPU box: fp32 + bf16 extraction bench lines and
# PMC passes over layer3's 3x3 forward k-loop (fill on / off).
# usage: bash tools/gpu_r3_extra.sh  -> gpurun_out/r3extra/
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r3extra
mkdir -p $o
timeout -k 10 300 python bench.py --workload extract --dtype fp32 --steps 20 > $o/extract_fp32.log 2>&1 || { tail -5 $o/extract_fp32.log; exit 1; }
tail -1 $o/extract_fp32.log | cut -c1-200
timeout -k 10 300 python bench.py --workload extract --steps 20 > $o/extract_bf16.log 2>&1 || { tail -5 $o/extract_bf16.log; exit 1; }
tail -1 $o/extract_bf16.log | cut -c1-200
for d in 0 3; do
  for f in 256,256,4,2,2 128,128,4,2,2; do
    tag=d${d}_${f//,/x}
    SSIP_DIAG=$d SSIP_CONV_FORCE=f,$f timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES \
      --output-format csv -d $o/p1_$tag -o run -- python tools/pmc_conv_loop.py > $o/p1_$tag.log 2>&1 || { tail -5 $o/p1_$tag.log; exit 1; }
    SSIP_DIAG=$d SSIP_CONV_FORCE=f,$f timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
      --output-format csv -d $o/p2_$tag -o run -- python tools/pmc_conv_loop.py > $o/p2_$tag.log 2>&1 || { tail -5 $o/p2_$tag.log; exit 1; }
  done
done
echo "r3extra done"
