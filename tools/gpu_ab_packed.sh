# A/B of prebuilt library variants (variants/NAME/libtdstar.so) on the two-chains-per-CU leg: 512 config-3
# chains in the tiles-in-LDS 4-wave kernel (lds_mode 2), stamped phases, each variant twice interleaved.
# usage: tools/gpu_ab_packed.sh TAG NAME...
set -o pipefail
O=gpurun_out/$1; shift
mkdir -p $O
for rep in 1 2; do
  for v in "$@"; do
    TD_LIB_PATH=$PWD/variants/$v/libtdstar.so TD_LDS_MODE=${TD_LDS_MODE:-2} timeout -k 10 200 python tools/batch_phases.py 512 2000 > $O/$v.$rep.json 2>&1 || { echo "$v failed"; tail $O/$v.$rep.json; exit 1; }
    python3 -c "
import json;d=json.load(open('$O/$v.$rep.json'));print('$v',$rep,round(d['proposals_per_s']/1e6,2),'M/s',d['total'],d['cycles_per_iter_per_chain'],d['F per wave'][:4])"
  done
done
