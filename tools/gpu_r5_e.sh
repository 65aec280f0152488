#!/bin/bash
# GPU box (round 5): s_setprio 1 for the second half of 8/16-wave workgroups (tools/lab/prio build)
# vs the default build: per-launch conv times, halo lab, step A/B.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
o=gpurun_out/r5e
mkdir -p $o
P=$R/tools/lab/prio/libssip_hip.so
D=$R/semi-supervised-image-processing_amd/ssip/libssip_hip.so
for v in def prio def2 prio2; do
  case $v in def*) L=$D;; *) L=$P;; esac
  SSIP_LIB=$L timeout -k 10 300 python -u tools/conv_times.py > $o/conv_$v.log 2>&1 || { echo conv_times failed; tail -5 $o/conv_$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $o/conv_$v.log
done
bash tools/ab_env.sh prio "SSIP_LIB=$D" "SSIP_LIB=$P" 2 || exit 1
