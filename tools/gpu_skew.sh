# The chain's wave-skew check (chain_kernels.hip SKEW, make skew-lib): the chain, bench-parity and
# drop-in tests on skew builds, each named on the command line as name=path.so.
#   bash tools/gpu_skew.sh OUT name=ab/libtdstar_skew_new.so [name2=...]
# A build's failures are recorded, not fatal (an old build may be expected to fail); a time limit is.
set -o pipefail
out=gpurun_out/$1; shift
mkdir -p $out
T="tests/test_gpu_chain.py tests/test_gpu_bench_parity.py tests/test_gpu_incremental.py"
for nv in "$@"; do
  v=${nv%%=*}; lib=${nv#*=}
  export TD_LIB_PATH=$PWD/$lib
  timeout -k 10 900 python -u -m pytest $T -v -p no:cacheprovider --timeout 150 --timeout-method thread --durations 15 \
    -k "not do_not_hold_back" > $out/$v.log 2>&1
  rc=$?
  echo "$v rc=$rc: $(tail -1 $out/$v.log)"
  unset TD_LIB_PATH
  if [ $rc -ge 124 ]; then echo "time limit: stopping"; exit 1; fi
done
