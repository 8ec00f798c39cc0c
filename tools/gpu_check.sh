set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_posterior.py -x -q > gpurun_out/t_post.log 2>&1 || { echo "posterior tests failed"; exit 1; }
