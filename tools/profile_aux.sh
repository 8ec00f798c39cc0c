#!/bin/bash
# rocprofv3 evidence for SURVEY 8f rows 2 and 4 (posterior section, trilinear
# slowness) and the full evaluate: kernel trace + stats, then one PMC pass per
# counter group (never combined with a trace domain).  usage: tools/profile_aux.sh TAG
set -o pipefail
TAG=${1:-aux}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG/aux
mkdir -p $OUT
A="--steps 1 --warmup 0 --no-cpu-baseline --no-dropin --no-config4 --no-stress --batch-chains 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $A > $OUT/trace.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py $A > $OUT/fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py $A > $OUT/write.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o run -- python3 bench.py $A > $OUT/sq.log 2>&1 || exit 1
