# same-box A/B of the many-chain rates (256 chains one per CU, 512 two per CU) over several builds,
# interleaved twice:  bash tools/gpu_many_ab.sh OUT name=path.so ... (an empty path = the working tree's build)
set -o pipefail
out=gpurun_out/$1; shift
mkdir -p $out
A="--steps 2 --warmup 1 --no-cpu-baseline --no-full-evaluate --no-dropin --no-config4 --no-stress --no-phases"
for k in 1 2; do
  for nv in "$@"; do
    v=${nv%%=*}; lib=${nv#*=}
    if [ -n "$lib" ]; then export TD_LIB_PATH=$PWD/$lib; else unset TD_LIB_PATH; fi
    timeout -k 10 240 python bench.py $A > $out/$v$k.json 2>&1 || { echo "$v failed"; tail $out/$v$k.json; exit 1; }
    python -c "
import json; d=json.loads(open('$out/$v$k.json').read().strip().splitlines()[-1])
m, p = d['many_chains'], d['many_chains_2per_cu']
print('$v', d['value'], m['proposals_per_s'], p['proposals_per_s'], m['ms_per_launch'], p['ms_per_launch'])"
  done
done
