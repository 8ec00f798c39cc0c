set -o pipefail
mkdir -p gpurun_out
export TD_BENCH_BACKEND=gloo TD_BENCH_DEVICE=0
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --batch-chains 0 --no-stress --no-full-evaluate > gpurun_out/bench_n2.log 2>&1 || { echo "n2 failed"; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --batch-chains 0 --no-stress --no-full-evaluate --chains-per-gpu 2 --swap-every 500 > gpurun_out/bench_n2t.log 2>&1 || { echo "n2 tempering failed"; exit 1; }
