# tempering mixing statistics: the ladder tests, then the default bench and the 2-rank gloo rehearsal
set -e
mkdir -p gpurun_out/mix
timeout -k 10 400 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_config4.py tests/test_gpu_bench_ranks.py tests/test_tempering.py -k "temper or config4 or ranks or round_trip" -x -v --timeout 300 --timeout-method thread > gpurun_out/mix/t.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/mix/bench.log 2>&1
TD_BENCH_BACKEND=gloo TD_BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/mix/bench2.log 2>&1
