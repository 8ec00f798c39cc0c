# round-end check: all GPU tests, smoke, the default bench line
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/final_tests.log 2>&1
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/final_bench.log 2>&1
# the N > 1 path rehearsed on one GPU: two ranks, gloo, both on device 0
TD_BENCH_BACKEND=gloo TD_BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/final_bench2.log 2>&1
