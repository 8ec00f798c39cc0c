# same-box A/B of the headline chain over several builds, interleaved twice:
#   bash tools/gpu_ab.sh OUT name=path.so ... (an empty path = the working tree's libtdstar.so)
# then the chain parity tests on the working tree (skip with TESTS=0)
set -o pipefail
out=gpurun_out/$1; shift
mkdir -p $out
A="--steps 10 --warmup 2 --no-cpu-baseline --no-full-evaluate --no-dropin --no-config4 --no-stress --batch-chains 0"
for k in 1 2; do
  for nv in "$@"; do
    v=${nv%%=*}; lib=${nv#*=}
    if [ -n "$lib" ]; then export TD_LIB_PATH=$PWD/$lib; else unset TD_LIB_PATH; fi
    timeout -k 10 120 python bench.py $A > $out/$v$k.json 2>&1 || { echo "$v failed"; tail $out/$v$k.json; exit 1; }
    python -c "import json,sys; d=json.loads(open('$out/$v$k.json').read().strip().splitlines()[-1]); print('$v', d['value'], json.dumps(d['roofline']['latency']['phases']))"
  done
done
unset TD_LIB_PATH
[ "${TESTS:-1}" = 0 ] && exit 0
timeout -k 10 900 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_bench_parity.py tests/test_gpu_incremental.py -x -q --timeout 600 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests failed"; tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
