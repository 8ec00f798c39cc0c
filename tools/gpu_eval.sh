set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/t_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/t_gpu.log; exit 1; }
timeout -k 10 600 python bench.py --steps 3 --no-cpu-baseline --batch-chains 0 > gpurun_out/bench_fe.log 2>&1 || { echo "bench failed"; exit 1; }
timeout -k 10 120 python tools/eval_trace.py > gpurun_out/evt.log 2>&1 || { echo "eval trace failed"; exit 1; }
