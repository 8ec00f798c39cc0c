# same-box A/B of td_evaluate (bench.py's full_evaluate block: grid and brute force) over two builds, then the
# evaluate parity tests:  bash tools/gpu_eval_ab.sh OUT [base.so]   (base default ab/libtdstar_base.so)
set -o pipefail
out=gpurun_out/${1:-eab}; mkdir -p $out
BASE=${2:-ab/libtdstar_base.so}
A="--steps 1 --warmup 0 --iters-per-step 500 --no-cpu-baseline --no-dropin --no-config4 --no-stress --batch-chains 0 --no-phases"
for k in 1 2; do
  for v in base head; do
    if [ $v = base ]; then export TD_LIB_PATH=$PWD/$BASE; else unset TD_LIB_PATH; fi
    timeout -k 10 240 python bench.py $A > $out/$v$k.json 2>&1 || { echo "$v failed"; tail $out/$v$k.json; exit 1; }
    python -c "import json; d=json.loads(open('$out/$v$k.json').read().strip().splitlines()[-1]); f=d['full_evaluate']; print('$v', json.dumps({m: [f[m]['evaluate_ms'], f[m]['kernel_ms'], f[m]['host_us']] for m in ('grid', 'brute_force')}))"
  done
done
unset TD_LIB_PATH
timeout -k 10 600 python -u -m pytest tests/test_gpu_evaluate.py tests/test_gpu_kat.py tests/test_gpu_incremental.py tests/test_gpu_main.py -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo tests failed; tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
