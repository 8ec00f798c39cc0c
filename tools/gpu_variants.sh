# one test selection (-k EXPR) on several builds: bash tools/gpu_variants.sh OUT "EXPR" name=lib.so ...
set -o pipefail
out=gpurun_out/$1; shift
expr=$1; shift
mkdir -p $out
for nv in "$@"; do
  v=${nv%%=*}; lib=${nv#*=}
  if [ -n "$lib" ]; then export TD_LIB_PATH=$PWD/$lib; else unset TD_LIB_PATH; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_bench_parity.py -v -p no:cacheprovider \
    --timeout ${PT:-120} --timeout-method thread -k "$expr" > $out/$v.log 2>&1
  rc=$?
  echo "$v rc=$rc: $(tail -1 $out/$v.log)"
  if [ $rc -ge 124 ]; then echo "time limit: stopping"; exit 1; fi
done
