set -o pipefail
mkdir -p gpurun_out/fused
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_resnet.py -x -q --timeout 200 --timeout-method thread -k "dgrad_bn or fused_bn" > gpurun_out/fused/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/fused/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_env.sh fusemode "SSIP_FUSE_BN_BWD=0" "SSIP_FUSE_BN_BWD=" 3 && bash tools/ab_env.sh fusemode2 "SSIP_FUSE_BN_BWD=0" "SSIP_FUSE_BN_BWD=halo" 2
