# round-3 check: all GPU tests, smoke, the default bench line.  usage: tools/gpu_r3.sh TAG
set -o pipefail
TAG=${1:-r3}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { echo bench failed; tail $O/bench.log; exit 1; }
cat $O/smoke.log; tail -c 3000 $O/bench.log
