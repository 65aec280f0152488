export TMPDIR=/tmp
for v in "2048 4" "512 8" "1024 4" "256 8"; do
  set -- $v
  SSIP_BWD_BLOCKS=$1 SSIP_BWD_ITERS=$2 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/bnv_$1_$2 -o run -- python tools/time_bn_bwd.py > gpurun_out/bnv_$1_$2.log 2>&1 || exit 1
done
