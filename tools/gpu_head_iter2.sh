# chain iteration + the evaluate path's tests (ray sums shared)
set -e
bash tools/gpu_head_iter.sh
timeout -k 10 300 python -u -m pytest tests/test_gpu_evaluate.py tests/test_gpu_kat.py tests/test_gpu_sharded.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_eval.log 2>&1
