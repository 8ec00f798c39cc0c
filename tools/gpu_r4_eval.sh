# evaluate-path tests + the bench without the CPU leg
set -o pipefail
out=gpurun_out/${1:-r4e}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_evaluate.py tests/test_gpu_kat.py tests/test_gpu_incremental.py -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests failed"; tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 600 python bench.py --no-cpu-baseline > $out/bench.log 2>&1 || { echo bench failed; tail $out/bench.log; exit 1; }
tail -1 $out/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], json.dumps({k:(v['evaluate_ms'],v['kernel_ms'],v['host_us']) for k,v in d['full_evaluate'].items()}))"
