# A/B of the grid nearest search: quad-per-point (TD_NN_GRID_FORM=4) vs half-wave-per-point (TD_NN_GRID_FORM=1)
set -e
mkdir -p gpurun_out
TD_NN_GRID_FORM=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_evaluate.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gab_tests.log 2>&1
for i in 1 2; do
  for g in c3 stress; do
    a=""; if [ $g = stress ]; then a=stress; fi
    TD_NN_GRID_FORM=4 timeout -k 10 120 python tools/nn_grid_only.py $a 2 >> gpurun_out/gab_quad.log 2>&1
    TD_NN_GRID_FORM=1 timeout -k 10 120 python tools/nn_grid_only.py $a 2 >> gpurun_out/gab_half.log 2>&1
  done
done
