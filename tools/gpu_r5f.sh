# the drop-in server's phase stamps, then the default bench line (outputs under gpurun_out/$1)
set -o pipefail
out=gpurun_out/${1:-r5f}; mkdir -p $out
timeout -k 10 150 python tools/shadow_phases.py 1500 > $out/shadow.json || { echo shadow failed; exit 1; }
timeout -k 10 600 python bench.py > $out/bench.log 2>&1 || { echo bench failed; tail $out/bench.log; exit 1; }
tail -1 $out/bench.log | cut -c1-300
