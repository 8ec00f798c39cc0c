# the brute-force tile search and the posterior raster kernel: their GPU tests, then a profiled aux bench
set -o pipefail
O=gpurun_out/${1:-nnr}
mkdir -p $O/aux
[ -n "$NOTEST" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_evaluate.py tests/test_gpu_posterior.py -x -v --timeout 400 --timeout-method thread > $O/t.log 2>&1 || { echo "tests failed"; tail -50 $O/t.log; exit 1; }
[ -n "$NOTEST" ] || tail -3 $O/t.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A="--steps 1 --warmup 0 --no-cpu-baseline --no-dropin --no-config4 --batch-chains 0 --stress-iters 10"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/aux/trace -o run -- python3 bench.py $A > $O/aux/trace.log 2>&1 || { echo trace failed; tail $O/aux/trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/aux/fetch -o run -- python3 bench.py $A > $O/aux/fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/aux/write -o run -- python3 bench.py $A > $O/aux/write.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/aux/sq -o run -- python3 bench.py $A > $O/aux/sq.log 2>&1 || exit 1
python3 profiles/summarize.py $O/aux > $O/aux.md
tail -c 2500 $O/aux/trace.log | grep -o '"stress".*' | head -c 1500
