set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_exact_sum.py -x -q > gpurun_out/t_exact.log 2>&1 || { echo "exact tests failed"; exit 1; }
timeout -k 10 600 python -m pytest tests/test_gpu_evaluate.py -x -q > gpurun_out/t_eval.log 2>&1 || { echo "evaluate tests failed"; exit 1; }
timeout -k 10 600 python -m pytest tests/test_gpu_chain.py -x -q > gpurun_out/t_chain.log 2>&1 || { echo "chain tests failed"; exit 1; }
timeout -k 10 400 python bench.py --steps 3 --no-cpu-baseline --batch-chains 0 > gpurun_out/bench.log 2>&1 || { echo "bench failed"; exit 1; }
