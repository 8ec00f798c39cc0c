set -o pipefail
out=gpurun_out/${1:-r5g}
mkdir -p $out

timeout -k 10 900 python -u -m pytest tests/test_gpu_evaluate.py tests/test_gpu_kat.py tests/test_gpu_incremental.py tests/test_gpu_main.py -x -q --timeout 600 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests failed"; tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-dropin --no-config4 --batch-chains 0 --no-phases > $out/bench.log 2>&1 || { tail $out/bench.log; exit 1; }
python -c "
import json
d=json.loads(open('$out/bench.log').read().strip().splitlines()[-1])
print(json.dumps(d['full_evaluate']['grid'])); print(json.dumps(d['stress']['evaluate']['grid']))
"
