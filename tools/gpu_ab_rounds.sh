# A/B of prebuilt library variants (variants/NAME/libtdstar.so) on BASELINE config 4's resident tempering
# rounds (tools/rounds_handshake.py: 1 and 8 replicas, K = 1 and 10), each variant twice interleaved.
# usage: tools/gpu_ab_rounds.sh TAG NAME...
set -o pipefail
O=gpurun_out/$1; shift
mkdir -p $O
for rep in 1 2; do
  for v in "$@"; do
    TD_LIB_PATH=$PWD/variants/$v/libtdstar.so TD_ROUNDS_TRACE=1 timeout -k 10 200 python tools/rounds_handshake.py 300 > $O/$v.$rep.log 2>&1 || { echo "$v failed"; tail $O/$v.$rep.log; exit 1; }
    echo "$v $rep $(grep -E '^\{"R8_K10' $O/$v.$rep.log) $(grep rounds_trace $O/$v.$rep.log | tail -1)"
  done
done
