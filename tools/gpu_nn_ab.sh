set -o pipefail
mkdir -p gpurun_out/nn1
for k in 1 2; do
  TD_LIB_PATH=$PWD/ab/libtdstar_base.so timeout -k 10 120 python tools/nn_tile_ppl.py > gpurun_out/nn1/base$k.json 2>&1 || { tail gpurun_out/nn1/base$k.json; exit 1; }
  timeout -k 10 120 python tools/nn_tile_ppl.py > gpurun_out/nn1/head$k.json 2>&1 || { tail gpurun_out/nn1/head$k.json; exit 1; }
  echo base; tail -1 gpurun_out/nn1/base$k.json; echo head; tail -1 gpurun_out/nn1/head$k.json
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_evaluate.py tests/test_gpu_kat.py tests/test_gpu_incremental.py -x -q --timeout 300 --timeout-method thread > gpurun_out/nn1/tests.log 2>&1 || { tail -30 gpurun_out/nn1/tests.log; exit 1; }
tail -2 gpurun_out/nn1/tests.log
