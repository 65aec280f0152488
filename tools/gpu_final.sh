set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/final
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/pytest.log 2>&1; echo "pytest rc $?"; tail -2 $o/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1; echo "smoke rc $?"; tail -2 $o/smoke.log
timeout -k 10 420 python bench.py > $o/bench.log 2>&1; echo "bench rc $?"; tail -1 $o/bench.log
