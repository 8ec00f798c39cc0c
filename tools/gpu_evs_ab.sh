# The resident full evaluate's timing (tools/eval_server_time.py) for library / environment variants:
#   bash tools/gpu_evs_ab.sh OUT name=lib.so[:ENV=V] ...   (lib "-": the in-tree build)
set -o pipefail
out=gpurun_out/$1; shift
mkdir -p $out
for nv in "$@"; do
  v=${nv%%=*}; rest=${nv#*=}; lib=${rest%%:*}; envs=""
  [ "$rest" != "$lib" ] && envs=${rest#*:}
  if [ "$lib" = "-" ]; then unset TD_LIB_PATH; else export TD_LIB_PATH=$PWD/$lib; fi
  env $envs timeout -k 10 120 python -u tools/eval_server_time.py 300 > $out/$v.json 2> $out/$v.err
  rc=$?
  echo "$v rc=$rc"; cat $out/$v.json
  if [ $rc -ne 0 ]; then exit 1; fi
done
