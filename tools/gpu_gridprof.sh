# counter passes of the bucket-grid nearest search (tools/nn_grid_only.py): config 3 and stress
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/gridprof
mkdir -p $O
for g in c3 stress; do
  a=""; if [ $g = stress ]; then a=stress; fi
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $O/${g}_trace -o run -- python3 tools/nn_grid_only.py $a 2 > $O/${g}_trace.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_WAIT_ANY -d $O/${g}_p1 -o run -- python3 tools/nn_grid_only.py $a 2 > $O/${g}_p1.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE FETCH_SIZE SQ_INST_CYCLES_VMEM SQ_LEVEL_WAVES -d $O/${g}_p2 -o run -- python3 tools/nn_grid_only.py $a 2 > $O/${g}_p2.log 2>&1
done
