set -o pipefail
mkdir -p gpurun_out/r1s3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r1s3/tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r1s3/tests.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1s3/smoke.log 2>&1 || { echo smoke failed; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/r1s3/bench.log 2>&1 || { echo bench failed; tail gpurun_out/r1s3/bench.log; exit 1; }
tail -3 gpurun_out/r1s3/tests.log; cat gpurun_out/r1s3/smoke.log; tail -2 gpurun_out/r1s3/bench.log
