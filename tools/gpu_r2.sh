# round-2 GPU check: the given test files first, then the whole GPU suite, smoke and a short bench
# usage: tools/gpu_r2.sh OUTDIR [test files...]
set -o pipefail
O=gpurun_out/${1:-r2}; shift
mkdir -p $O
if [ $# -gt 0 ]; then
timeout -k 10 600 python -u -m pytest "$@" -x -v --timeout 400 --timeout-method thread > $O/new.log 2>&1 || { echo "new tests failed"; tail -60 $O/new.log; exit 1; }
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/tests.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
timeout -k 10 600 python bench.py --steps 5 --cpu-seconds 4 > $O/bench.log 2>&1 || { echo bench failed; tail $O/bench.log; exit 1; }
tail -5 $O/new.log 2>/dev/null; tail -3 $O/tests.log; cat $O/smoke.log; tail -c 1500 $O/bench.log
