# counter passes of the tile nearest search alone (tools/nn_tile_only.py, config-3 points x 5000 cells)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/nnprof
mkdir -p $O
timeout -s KILL 60 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 tools/nn_tile_only.py 5000 200 > $O/trace.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_WAIT_ANY -d $O/p1 -o run -- python3 tools/nn_tile_only.py 5000 200 > $O/p1.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY -d $O/p2 -o run -- python3 tools/nn_tile_only.py 5000 200 > $O/p2.log 2>&1
