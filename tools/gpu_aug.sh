set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/aug
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_augment.py -x -q --timeout 300 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -2 $o/pytest.log
for v in 1 4 8; do
  SSIP_AUG_ROWS=$v timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $o/tr$v -o run -- python bench.py --steps 5 --warmup 3 --no-cpu-baseline --exec eager > $o/tr$v.log 2>&1 || exit 1
done
bash tools/ab_env.sh aug/ab 3 "SSIP_AUG_ROWS=1" "SSIP_AUG_ROWS=4"
