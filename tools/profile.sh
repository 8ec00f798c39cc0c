#!/bin/bash
# rocprofv3 evidence for profiles/: kernel trace + stats, then one PMC pass per
# counter group (never combined with any trace domain).  usage: tools/profile.sh TAG
set -o pipefail
TAG=${1:-prof}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p $OUT
run() {  # name, bench args...
    local name=$1; shift
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$name/trace -o run -- python3 bench.py "$@" > $OUT/$name/trace.log 2>&1 || return 1
    timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/$name/fetch -o run -- python3 bench.py "$@" > $OUT/$name/fetch.log 2>&1 || return 1
    timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/$name/write -o run -- python3 bench.py "$@" > $OUT/$name/write.log 2>&1 || return 1
    timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/$name/sq -o run -- python3 bench.py "$@" > $OUT/$name/sq.log 2>&1 || return 1
}
trace_only() {  # name, bench args...: kernel trace only (PMC passes serialize the dispatches: the exchange
    local name=$1; shift  # rounds' resident kernel and RCCL's allgather kernels must run side by side)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$name/trace -o run -- python3 bench.py "$@" > $OUT/$name/trace.log 2>&1 || return 1
}
mkdir -p $OUT/single $OUT/many $OUT/packed $OUT/stress $OUT/config4
if [ -n "$2" ]; then  # one pass only: tools/profile.sh TAG stress
    [ "$2" = stress ] && { run stress --steps 1 --warmup 0 --iters-per-step 10 --no-cpu-baseline --no-full-evaluate --no-dropin --no-config4 --batch-chains 0 || exit 1; }
    [ "$2" = single ] && { run single --steps 3 --warmup 1 --no-cpu-baseline --batch-chains 0 --no-stress --no-dropin --no-config4 || exit 1; }
    exit 0
fi
run single --steps 3 --warmup 1 --no-cpu-baseline --batch-chains 0 --no-stress --no-dropin --no-config4 && \
run many --steps 2 --warmup 1 --no-cpu-baseline --no-full-evaluate --no-dropin --no-config4 --no-stress --batch-chains 0 --chains-per-gpu 256 --iters-per-step 5000 && \
run packed --steps 1 --warmup 0 --iters-per-step 10 --no-cpu-baseline --no-full-evaluate --no-dropin --no-config4 --no-stress --batch-chains 256 --batch-iters 5000 && \
run stress --steps 1 --warmup 0 --iters-per-step 10 --no-cpu-baseline --no-full-evaluate --no-dropin --no-config4 --batch-chains 0 && \
trace_only config4 --steps 1 --warmup 0 --iters-per-step 10 --no-cpu-baseline --no-full-evaluate --no-dropin --no-stress --batch-chains 0
