# exchange rounds: the new GPU tests (one-rank device swaps, lone RCCL comm, RCCL world 1 under torch.distributed.run)
set -o pipefail
out=gpurun_out/${1:-r4x}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -v -s --timeout 120 --timeout-method thread -k "exchange or hold_back or partial" > $out/chain.log 2>&1 || { echo "chain tests failed"; tail -40 $out/chain.log; exit 1; }
tail -3 $out/chain.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_config4.py -x -v -s --timeout 400 --timeout-method thread > $out/c4.log 2>&1 || { echo "config4 tests failed"; tail -60 $out/c4.log; exit 1; }
grep "rccl world 1" $out/c4.log | cut -c1-3000; tail -3 $out/c4.log
