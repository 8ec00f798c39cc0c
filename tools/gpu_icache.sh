# instruction-cache counters of the headline chain for several builds (rocprofv3 PMC, one pass each)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-icache}; shift
mkdir -p $out
timeout -k 5 60 rocprofv3 -L > $out/counters.txt 2>&1 || true
grep -i "icache\|SQC_\|IFETCH" $out/counters.txt | head -60 > $out/counters_sqc.txt || true
A="--steps 2 --warmup 1 --no-cpu-baseline --no-full-evaluate --no-dropin --no-config4 --no-stress --batch-chains 0 --no-phases"
for nv in "$@"; do
  v=${nv%%=*}; lib=${nv#*=}
  if [ -n "$lib" ]; then export TD_LIB_PATH=$PWD/$lib; else unset TD_LIB_PATH; fi
  timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY --output-format csv -d $out/$v -o run -- python3 bench.py $A > $out/$v.log 2>&1 || { echo "$v failed"; tail -5 $out/$v.log; }
done
