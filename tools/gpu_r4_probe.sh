# quick probes: mailbox latency placements, then the default bench without the CPU leg
set -o pipefail
out=gpurun_out/${1:-r4p}
mkdir -p $out
timeout -k 10 60 ./tools/mailbox_latency > $out/mailbox.log 2>&1; echo "mailbox rc=$?"; cat $out/mailbox.log
timeout -k 10 600 python bench.py --no-cpu-baseline > $out/bench.log 2>&1 || { echo bench failed; tail $out/bench.log; exit 1; }
tail -1 $out/bench.log | cut -c1-300
