# the evaluate path alone, twice (same box), then its GPU tests
set -o pipefail
for k in 1 2; do timeout -k 10 120 python tools/eval_ab.py 300 || exit 1; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_evaluate.py tests/test_gpu_kat.py -x -q --timeout 300 --timeout-method thread 2>&1 | tail -2
