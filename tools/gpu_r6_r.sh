#!/bin/bash
# GPU box (round 6): where the layer-1 halo forward's time goes -- ablations at
# batch 256 and PMC passes (LDS, wait states, MFMA) on the full kernel and its no-math form.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6r
mkdir -p $o
timeout -k 10 300 python -u tools/halo_lab.py --batches 256 --diags 0,1,2,3,4,7,8,11,15 > $o/halo.log 2>&1 || { tail -5 $o/halo.log; exit 1; }
grep -v amdgpu.ids $o/halo.log | grep -v "stem\|pooled"
for dg in 0 3 15; do
  SSIP_HALO_DIAG=$dg timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --output-format csv -d $o/p1_$dg -o pmc -- \
    python3 tools/one_conv.py l1.3x3 f 10 > $o/p1_$dg.log 2>&1 || { tail -5 $o/p1_$dg.log; exit 1; }
  python3 tools/pmc_kernel_sum.py $(find $o/p1_$dg -name "*counter_collection.csv" | head -1) conv_halo "diag $dg"
  SSIP_HALO_DIAG=$dg timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU \
    GRBM_GUI_ACTIVE --output-format csv -d $o/p2_$dg -o pmc -- \
    python3 tools/one_conv.py l1.3x3 f 10 > $o/p2_$dg.log 2>&1 || { tail -5 $o/p2_$dg.log; exit 1; }
  python3 tools/pmc_kernel_sum.py $(find $o/p2_$dg -name "*counter_collection.csv" | head -1) conv_halo "diag $dg"
done
SSIP_HALO_DIAG=0 timeout -s KILL 60 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU \
  SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_MFMA --output-format csv -d $o/p3_0 -o pmc -- \
  python3 tools/one_conv.py l1.3x3 f 10 > $o/p3_0.log 2>&1 && \
  python3 tools/pmc_kernel_sum.py $(find $o/p3_0 -name "*counter_collection.csv" | head -1) conv_halo "diag 0"
echo "r6r done"
