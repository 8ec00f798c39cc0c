# quick GPU iteration: the given tests, then the drop-in bench leg
set -o pipefail
O=gpurun_out/${1:-q}; shift
mkdir -p $O
timeout -k 10 600 python -u -m pytest "$@" -x -q --timeout 400 --timeout-method thread > $O/t.log 2>&1 || { echo "tests failed"; tail -50 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 300 python tools/dropin_only.py > $O/dropin.log 2>&1 || { echo dropin failed; tail $O/dropin.log; exit 1; }
cat $O/dropin.log
