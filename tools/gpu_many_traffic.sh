# PMC HBM traffic of the 256-chain launch (one chain per CU) for several builds, one counter per pass:
#   bash tools/gpu_many_traffic.sh OUT name=path.so ...   (summarise with tools/many_traffic.py OUT)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$1; shift
A="--steps 2 --warmup 1 --no-cpu-baseline --no-full-evaluate --no-dropin --no-config4 --no-stress --no-phases --batch-chains 0 --chains-per-gpu 256 --iters-per-step 5000"
for nv in "$@"; do
  v=${nv%%=*}; lib=${nv#*=}
  if [ -n "$lib" ]; then export TD_LIB_PATH=$PWD/$lib; else unset TD_LIB_PATH; fi
  mkdir -p $out/$v
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $out/$v/$c -o run -- python3 bench.py $A > $out/$v/$c.log 2>&1 || { echo "$v $c failed"; tail $out/$v/$c.log; exit 1; }
  done
  echo "$v done"
done
