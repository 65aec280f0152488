set -o pipefail
mkdir -p gpurun_out/abfuse
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/abfuse/a$i.log 2>&1 || exit 1
  SSIP_FUSE_BN_BWD=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/abfuse/b$i.log 2>&1 || exit 1
done
for f in gpurun_out/abfuse/*.log; do echo $f $(grep -o '"ms_per_step": [0-9.]*' $f); done
