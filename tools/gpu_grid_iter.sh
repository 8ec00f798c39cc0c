# grid search: evaluate tests + the search alone at config 3 and stress
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_evaluate.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_eval.log 2>&1
for i in 1 2; do
  timeout -k 10 120 python tools/nn_grid_only.py >> gpurun_out/grid_it.log 2>&1
  timeout -k 10 120 python tools/nn_grid_only.py stress >> gpurun_out/grid_it.log 2>&1
done
