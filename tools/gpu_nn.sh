# brute-force nearest iteration: parity tests, the search alone over cell counts, time(N) scan
set -o pipefail
O=gpurun_out/${1:-nn}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_evaluate.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { echo "tests failed"; tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 200 python tools/nn_bench2.py > $O/b2.log 2>&1 || { echo bench2 failed; tail $O/b2.log; exit 1; }
cat $O/b2.log
timeout -k 10 200 python tools/nn_scan.py > $O/scan.log 2>&1 || { echo scan failed; tail $O/scan.log; exit 1; }
cat $O/scan.log
