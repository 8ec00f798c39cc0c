set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_evaluate.py tests/test_gpu_chain.py -x -q > gpurun_out/t_all.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --batch-chains 0 > gpurun_out/bench.log 2>&1 || { echo "bench failed"; exit 1; }
