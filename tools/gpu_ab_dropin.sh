# A/B of prebuilt library variants (variants/NAME/libtdstar.so) on bench.py's drop-in leg (an unchanged
# host's td_evaluate per proposal through the resident server), each variant twice interleaved.
# usage: tools/gpu_ab_dropin.sh TAG NAME...
set -o pipefail
O=gpurun_out/$1; shift
mkdir -p $O
for rep in 1 2; do
  for v in "$@"; do
    TD_LIB_PATH=$PWD/variants/$v/libtdstar.so timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-full-evaluate --no-config4 --no-stress --batch-chains 0 --no-phases > $O/$v.$rep.bench 2>&1 || { echo "$v bench failed"; tail $O/$v.$rep.bench; exit 1; }
    python3 -c "import json;b=json.loads([l for l in open('$O/$v.$rep.bench') if l.startswith('{')][-1]);print('$v',$rep,b['dropin']['incremental'])"
  done
done
