# round 6 check: chain tests on one build (TD_LIB_PATH, default the in-tree one), then a headline A/B
#   bash tools/gpu_r6.sh OUT [lib.so|-] name=lib.so ...
set -o pipefail
out=gpurun_out/$1; shift
first=$1; shift
mkdir -p $out
if [ "$first" != "-" ]; then export TD_LIB_PATH=$PWD/$first; fi
if [ -z "$NOTESTS" ]; then
timeout -k 10 800 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_bench_parity.py tests/test_gpu_evaluate.py tests/test_gpu_kat.py tests/test_gpu_incremental.py -v -x -p no:cacheprovider \
  --timeout 150 --timeout-method thread --durations 10 > $out/tests.log 2>&1
rc=$?
unset TD_LIB_PATH
echo "tests rc=$rc: $(tail -1 $out/tests.log)"
[ $rc -ne 0 ] && { grep -E "FAILED|Error|Timeout" $out/tests.log | head -20; exit 1; }
fi
unset TD_LIB_PATH
A="--steps 10 --warmup 2 --no-cpu-baseline --no-full-evaluate --no-dropin --no-config4 --no-stress --batch-chains 0"
for k in 1 2; do
  for nv in "$@"; do
    v=${nv%%=*}; lib=${nv#*=}
    if [ -n "$lib" ]; then export TD_LIB_PATH=$PWD/$lib; else unset TD_LIB_PATH; fi
    timeout -k 10 120 python bench.py $A > $out/$v$k.json 2>&1 || { echo "$v failed"; tail $out/$v$k.json; exit 1; }
    python -c "import json,sys; d=json.loads(open('$out/$v$k.json').read().strip().splitlines()[-1]); print('$v', d['value'], json.dumps(d['roofline']['latency']['phases']))"
  done
done
