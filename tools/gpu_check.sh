# The round's full GPU check in one call: every GPU test, smoke, the default bench line
# (outputs under gpurun_out/$1)
set -o pipefail
out=gpurun_out/${1:-check}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $out/tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $out/tests.log; exit 1; }
tail -3 $out/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo smoke failed; cat $out/smoke.log; exit 1; }
timeout -k 10 600 python bench.py > $out/bench.log 2>&1 || { echo bench failed; tail $out/bench.log; exit 1; }
cat $out/smoke.log; tail -1 $out/bench.log | cut -c1-600
