# round-2 GPU check: new tests first, then the whole GPU suite, smoke and a short bench
set -o pipefail
O=gpurun_out/${1:-r2}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kat.py tests/test_gpu_config4.py -x -v --timeout 400 --timeout-method thread > $O/new.log 2>&1 || { echo "new tests failed"; tail -40 $O/new.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/tests.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
timeout -k 10 600 python bench.py --steps 5 --cpu-seconds 4 > $O/bench.log 2>&1 || { echo bench failed; tail $O/bench.log; exit 1; }
tail -3 $O/new.log; tail -3 $O/tests.log; cat $O/smoke.log; tail -c 3000 $O/bench.log
