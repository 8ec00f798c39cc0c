# sharded evaluate + misfit KAT + stress chain at 20k cells, then a 2-rank gloo rehearsal of bench.py on device 0
set -o pipefail
O=gpurun_out/${1:-shard}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_kat.py "tests/test_gpu_chain.py::test_stress_geometry_chain_follows_host_engine" -x -v --timeout 400 --timeout-method thread > $O/t.log 2>&1 || { echo "tests failed"; tail -40 $O/t.log; exit 1; }
tail -15 $O/t.log
TD_BENCH_BACKEND=gloo TD_BENCH_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --batch-chains 0 --no-config4 --no-dropin --no-full-evaluate > $O/bench2.log 2>&1 || { echo "bench2 failed"; tail -30 $O/bench2.log; exit 1; }
grep '^{' $O/bench2.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(json.dumps({k: d[k] for k in ('value','n_gpus','ms_per_step','stress_sharded') if k in d}))"
