# td_evaluate's kernels: PMC traffic (FETCH_SIZE, WRITE_SIZE: separate passes, no trace domains) of
# tools/eval_time.py per library variant, then the timing A/B and the evaluate parity tests
# (tools/gpu_eval_ab.sh).  usage: bash tools/gpu_eval_traffic.sh OUT name=lib.so ... ("-": in-tree)
set -o pipefail
tag=$1; out=gpurun_out/$1; shift
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for nv in "$@"; do
  v=${nv%%=*}; lib=${nv#*=}
  if [ "$lib" = "-" ]; then unset TD_LIB_PATH; else export TD_LIB_PATH=$PWD/$lib; fi
  mkdir -p $out/$v
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 120 rocprofv3 --pmc $c --output-format csv -d $out/$v/$c -o run -- python3 tools/eval_time.py 50 > $out/$v/$c.log 2>&1 || { echo "$v $c failed"; tail $out/$v/$c.log; exit 1; }
  done
done
unset TD_LIB_PATH
python3 tools/pmc_kernels.py $out "$@" || exit 1
bash tools/gpu_eval_ab.sh ${tag}_ab "$@"
