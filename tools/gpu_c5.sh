set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/c5
mkdir -p $o
timeout -k 10 500 python bench.py --arch resnet50 --image-size 512 --batch 128 --no-cpu-baseline > $o/c5.log 2>&1; echo "c5 rc $?"; tail -1 $o/c5.log
timeout -k 10 500 python bench.py --workload extract > $o/ex.log 2>&1; echo "ex rc $?"; tail -1 $o/ex.log
