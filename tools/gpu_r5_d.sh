#!/bin/bash
# GPU box (round 5): halo k-loop with per-step scheduling fences vs HEAD (ab_base).
# parity of the new build, halo lab + PMC for both libraries, step A/B.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
o=gpurun_out/r5d
mkdir -p $o
BASE=$R/ab_base/semi-supervised-image-processing_amd/ssip/libssip_hip.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_halo.py tests/test_gpu_conv.py tests/test_gpu_eval_fold.py tests/test_gpu_block_fusion.py \
  tests/test_gpu_resnet.py > $o/tests.log 2>&1 || { echo tests failed; tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
for v in new base; do
  if [ $v = base ]; then L=$BASE; else L=$R/semi-supervised-image-processing_amd/ssip/libssip_hip.so; fi
  SSIP_LIB=$L timeout -k 10 300 python -u tools/halo_lab.py --diags 0,4,8 > $o/halo_$v.log 2>&1 || { echo halo lab failed; tail -5 $o/halo_$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $o/halo_$v.log | grep -v "stem\|pooled"
  for m in f d; do
    SSIP_LIB=$L timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
      SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS -d $o/pmc1_${v}_$m -o pmc -- \
      python3 tools/one_conv.py l1.3x3 $m 10 > $o/pmc1_${v}_$m.log 2>&1 || { tail -5 $o/pmc1_${v}_$m.log; exit 1; }
    SSIP_LIB=$L timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE \
      -d $o/pmc2_${v}_$m -o pmc -- python3 tools/one_conv.py l1.3x3 $m 10 > $o/pmc2_${v}_$m.log 2>&1 || { tail -5 $o/pmc2_${v}_$m.log; exit 1; }
    for c in FETCH_SIZE WRITE_SIZE; do
      SSIP_LIB=$L timeout -s KILL 90 rocprofv3 --pmc $c \
        -d $o/pmc_${c}_${v}_$m -o pmc -- python3 tools/one_conv.py l1.3x3 $m 10 > $o/pmc_${c}_${v}_$m.log 2>&1 || { tail -5 $o/pmc_${c}_${v}_$m.log; exit 1; }
    done
  done
done
SSIP_HALO_DEFER=1 timeout -k 10 300 python -u tools/halo_lab.py --diags 0,4,8 > $o/halo_defer.log 2>&1 || { echo halo lab failed; tail -5 $o/halo_defer.log; exit 1; }
echo "== defer"; grep -v amdgpu.ids $o/halo_defer.log | grep -v "stem\|pooled"
bash tools/ab_env.sh fence "SSIP_LIB=$BASE" "SSIP_LIB=$R/semi-supervised-image-processing_amd/ssip/libssip_hip.so" 2 || exit 1
